"""bench.py's N > 1 path (the driver's multi-GPU scaling run) as the driver launches it: a fresh
`torch.distributed.run` child with two ranks, each on this box's one GPU, over gloo
(R3DG_DIST_BACKEND=gloo rehearses the RCCL path: same bench code, view-parallel exchange, barrier +
max-over-ranks timing). Rank 0's JSON line must carry the contract fields and the exchange
measurement (standalone collectives, compute-only step, exposed exchange time)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_gloo():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, R3DG_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--P", "20000",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=360)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["unit"] == "Mpix/s"
    assert abs(d["value"] - 2 * 1920 * 1080 / d["ms_per_step"] / 1e3) < 1e-3 * d["value"]
    ex = d["exchange"]
    assert ex["backend"] == "gloo"
    # the replayed sequence is the step's own: the camera-centre gather + 2 collectives per chunk
    # (4 chunks: 9), one packed 22-float all-reduce and one 3-float all-gather per Gaussian in total
    assert d["collectives_per_step"] == ex["collectives_per_step"] == 9
    assert ex["all_reduce"]["calls"] == 4 and ex["all_gather"]["calls"] == 5
    assert ex["all_reduce"]["bytes"] == 20000 * 22 * 4 and ex["all_reduce"]["ms"] > 0
    assert ex["all_gather"]["bytes_per_rank"] == (20000 * 3 + 3) * 4 and ex["all_gather"]["ms"] > 0
    assert ex["compute_only_ms_per_step"] > 0
    assert abs(ex["exposed_exchange_ms_per_step"] - (d["ms_per_step"] - ex["compute_only_ms_per_step"])) < 1e-3
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["binding"] and rf["extra_bytes"] == 12 * d["config"]["num_rendered"]
