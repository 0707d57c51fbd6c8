"""Benchmark of the hot path: rasterize_gaussians + rasterize_gaussians_backward (Mpix/s fwd+bwd).

Workload (BASELINE.json metric, SURVEY.md §8d "M1"): 1,000,000 synthetic Gaussians, 1920x1080,
S=11 features, SH degree 3, default shaders, pseudo normal on, backward_geometry on; upstream
gradients N(0,1)*1e-3 in the reference's CHW contract. One step = one view: the reference's
`_C.rasterize_gaussians` then `_C.rasterize_gaussians_backward` through this build's `_C`, and,
when N > 1, the per-Gaussian gradient exchange (view_parallel.py: RCCL all-reduce of means3D 3 + opacity 1 +
scales 3 + rotations 4 + features 11 floats, all-gather of each view's 3-float SH colour gradient,
the 48-float SH gradient sum rebuilt on every rank) -- view-parallel data parallelism, every rank
renders its own camera of the same scene (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Rank 0 prints one JSON line. `roofline` prices renderCUDA fwd + bwd -- render_fwd_glds_kernel and
render_bwd_glds_kernel with its atomic second stage (plus the sums' memset; row_sum_kernel instead
with the rows reduction, R3DG_BWD_REDUCE=rows) -- with SURVEY.md
§8d's algorithmic bytes exactly (272*L + 156*H*W + 16*tiles at S=11; the 12*L the forward also moves
for its fused per-tile depth sort is reported apart, as `extra_bytes`) over their device time, from HIP
events recorded inside each launch's dispatch on the launch stream during K further steps (the
timed K steps run without events);
`traffic` is the HBM bytes of the same kernels from rocprofv3 PMC counters (profiles/, FETCH_SIZE
doubled per MI355X_MICROARCH.md §HBM), or null; `roofline.valu` is the compute side: VALU
lane-instructions per second (PMC SQ_INSTS_VALU per launch, profiles/valu_latest.json) over the same
live launch times against the VALU issue peak, with the evaluated pixel x instance pairs. `cpu_baseline` times the CPU oracle (a scalar C port of the
reference path) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
P_M1, W_M1, H_M1, S_M1 = 1_000_000, 1920, 1080, 11


def algorithmic_bytes(L: int, npix: int, tiles: int, S: int) -> tuple[int, int]:
    """SURVEY.md §8d per-unit figures, nothing added: fwd L*(56+4S) + Npix*(40+4S) + 8T,
    bwd L*(84+8S) + Npix*(28+4S) + 8T."""
    fwd = L * (56 + 4 * S) + npix * (40 + 4 * S) + 8 * tiles
    bwd = L * (84 + 8 * S) + npix * (28 + 4 * S) + 8 * tiles
    return fwd, bwd


def fused_sort_bytes(L: int) -> int:
    """Bytes the forward blend moves beyond §8d: it also sorts its tiles (the binning's (depth, id)
    pairs read, 8 B, the sorted point_list written, 4 B per instance; render_fwd.hip)."""
    return 12 * L


def load_traffic() -> dict | None:
    path = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


# VALU issue peak, lane-instructions/s: 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz
# (MI355X_MICROARCH.md: a wave64 VALU op issues over 2 cycles; = the 157.3 TFLOP/s f32 vector peak / 2)
VALU_PEAK = 256 * 4 * 32 * 2.4e9


def load_valu(P: int) -> dict | None:
    """profiles/valu_latest.json (tools/make_valu.py): per launch of each blend kernel, the VALU
    wave-instructions (PMC SQ_INSTS_VALU, MFMA excluded) and the evaluated pixel x instance pairs E
    (R3DG_EXP_COUNT build: live wave-steps x 64 lanes)."""
    path = os.path.join(ROOT, "profiles", "valu_latest.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return d if d.get("config") == f"M1 P={P}" else None


def valu_roofline(v: dict | None, launch_ms: dict) -> dict | None:
    """The blend's compute bound (SURVEY.md §8d VALU cross-check): lane-instructions issued per
    second over the live launch time, against the VALU issue peak."""
    if not v:
        return None
    out = {"unit": "lane-instr/s", "peak": VALU_PEAK, "source": "profiles/valu_latest.json"}
    tot_i, tot_t = 0.0, 0.0
    for k in ("render_fwd", "render_bwd", "row_sum"):
        if k not in v or not launch_ms.get(k):
            continue
        t = launch_ms[k] / 1e3
        lanes = v[k]["valu_insts"] * 64
        ent = {"valu_insts": v[k]["valu_insts"], "achieved": lanes / t, "frac": round(lanes / t / VALU_PEAK, 4)}
        if v[k].get("evals"):
            ent["evals"] = v[k]["evals"]
            ent["ops_per_eval"] = round(lanes / v[k]["evals"], 2)
        out[k] = ent
        tot_i += lanes
        tot_t += t
    if tot_t > 0:
        out["achieved"] = tot_i / tot_t
        out["frac"] = round(tot_i / tot_t / VALU_PEAK, 4)
    return out


def binding(hbm_frac: float, valu: dict | None) -> str:
    """What binds the blend, from the measured fractions of the two peaks: the larger one when it
    exceeds 0.6, otherwise neither is saturated and the loop waits on latency (dependent LDS / exp
    chains, the batch barrier)."""
    vf = float(valu.get("frac", 0.0)) if valu else 0.0
    top, name = max((hbm_frac, "hbm"), (vf, "valu"))
    if top >= 0.6:
        return name
    return f"latency (hbm {hbm_frac:.2f}, valu {vf:.2f} of peak)"


def cpu_baseline(scene) -> dict:
    """The CPU oracle (scalar C port of the reference path, one thread) on one full M1 step: the
    1M-Gaussian scene at 1920x1080, preprocess + sort + blend fwd + bwd (~20 s)."""
    import oracle
    from relightable3dgaussian_amd import synthetic

    cam = synthetic.m1_camera(W_M1, H_M1)
    w, h = cam.width, cam.height
    rng = np.random.default_rng(1)
    dc = (rng.normal(size=(3, h, w)) * 1e-3).astype(np.float32)
    do = (rng.normal(size=h * w) * 1e-3).astype(np.float32)
    dd = (rng.normal(size=h * w) * 1e-3).astype(np.float32)
    df = (rng.normal(size=(S_M1, h, w)) * 1e-3).astype(np.float32)
    oracle.build()
    t0 = time.perf_counter()
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations)
    oracle.rasterize_backward(o, dc, do, dd, df)
    dt = time.perf_counter() - t0
    return {"value": round(w * h / dt / 1e6, 6), "unit": "Mpix/s", "cores": 1, "kind": "port",
            "sample": f"oracle/r3dg_oracle.c (scalar C port), one full M1 step (1M Gaussians, {w}x{h}): "
                      f"preprocess+sort+blend fwd+bwd, {dt:.1f} s"}


def brdf_c1(dev) -> dict:
    """north_star's CPU leg: the reference's pure-PyTorch render equation (restated in
    oracle/brdf_torch.py, pinned by tests/golden/brdf.npz) on SURVEY §8d config C1 (P = 10k,
    Ns = 24, eval), fwd and fwd+bwd (loss = sum pbr + sum diffuse_light), median of 5 after 1
    warmup, on this host's CPU share; next to this build's HIP kernels on the same inputs."""
    import torch

    from oracle import brdf_torch

    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores) or cores))
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    inp = brdf_torch.c1_inputs(10_000, seed=0)
    keys = ["base", "rough", "metal", "normals", "viewdirs", "incidents", "env", "visibility"]

    def cpu_fwd(grad):
        t = {k: v.clone().requires_grad_(grad) for k, v in inp.items()}
        pbr, ex = brdf_torch.rendering_equation(*[t[k] for k in keys], 24)
        if grad:
            (pbr.sum() + ex["diffuse_light"].sum()).backward()

    def med(fn, n=5):
        fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    cpu_f, cpu_fb = med(lambda: cpu_fwd(False)), med(lambda: cpu_fwd(True))
    torch.set_num_threads(prev)

    import relightable3dgaussian_amd as r3

    g = [inp[k].to(dev) for k in keys]
    ones = torch.ones(10_000, 3, device=dev)

    def gpu(grad):
        pbr, dirs, dl = r3._C.render_equation_forward(*g, 24, False, False)
        if grad:
            r3._C.render_equation_backward(*g, 24, dirs, ones, ones, False)

    def gmed(fn, n=20):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    return {"config": "C1: P=10000, Ns=24, eval, synthetic inputs (SURVEY §8d)", "cores": cores, "kind": "port",
            "cpu_fwd_ms": round(cpu_f, 3), "cpu_fwd_bwd_ms": round(cpu_fb, 3),
            "gpu_fwd_ms": round(gmed(lambda: gpu(False)), 4), "gpu_fwd_bwd_ms": round(gmed(lambda: gpu(True)), 4),
            "sample": "oracle/brdf_torch.py: PyTorch-CPU restatement of gaussian_renderer/neilf.py:437-519"}


def bvh_visibility(means3D, scales, rots, dev) -> dict:
    """The BVH visibility tracer on the M1 Gaussians: RayTracer build and
    trace_visibility of 10k rays (the lambda_visibility loss, neilf.py:323-348) and of one ray per
    Gaussian (finetune_visibility, gaussian_model.py:446-465), rays from Gaussian centres into the
    hemisphere of a random unit normal (M1 has no normals). Median of 5, HIP events."""
    import torch

    from relightable3dgaussian_amd.bvh import RayTracer

    P = means3D.shape[0]
    g = torch.Generator(device=dev).manual_seed(3)
    normals = torch.nn.functional.normalize(torch.randn(P, 3, device=dev, generator=g), dim=1)
    q = torch.nn.functional.normalize(rots, dim=1)
    w, x, y, z = q.unbind(1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                     2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                     2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).view(P, 3, 3)
    Sinv = R @ torch.diag_embed(1.0 / scales ** 2) @ R.transpose(1, 2)  # get_inverse_covariance
    cov_inv = Sinv[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].contiguous()
    opac = torch.full((P, 1), 0.5, device=dev)

    def med(fn, n=5):
        fn()
        ts = []
        for _ in range(n):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    res = {"gaussians": P, "build_ms": round(med(lambda: RayTracer(means3D, scales, rots)), 4)}
    rt = RayTracer(means3D, scales, rots)
    for R_, key in ((10000, "trace_10k"), (P, "trace_all")):
        idx = torch.randint(0, P, (R_,), device=dev, generator=g) if R_ < P else torch.arange(P, device=dev)
        o = means3D[idx].contiguous()
        d = torch.randn(R_, 3, device=dev, generator=g)
        d = torch.where(((d * normals[idx]).sum(1, keepdim=True) < 0), -d, d).contiguous()
        res[key + "_ms"] = round(med(lambda: rt.trace_visibility(o, d, means3D, cov_inv, opac, normals)), 4)
        res[key + "_mean_visibility"] = round(float(rt.trace_visibility(o, d, means3D, cov_inv, opac,
                                                                        normals)["visibility"].mean()), 4)
    return res


def comm_probe(seq: list, dev, world: int, backend: str, iters: int = 5) -> dict:
    """The exchange's collectives alone, outside the timed loop (DESIGN.md §6 cost model): the exact
    sequence one step issued (view_parallel.LAST_COLLECTIVES: the camera-centre all-gather, then per
    chunk the all-reduce of the chunk's packed dense rows -- 22 floats per Gaussian -- and the
    all-gather of its 3-float SH colour gradients), replayed back to back on the current stream.
    Mean over `iters` after one warmup, barrier-bracketed, max over ranks. Bus bandwidth as
    nccl-tests defines it: all-reduce 2(N-1)/N * bytes / t, all-gather (N-1)/N * N * bytes / t."""
    import torch
    import torch.distributed as dist

    bufs = []
    for kind, n in seq:
        if kind == "all_reduce":
            bufs.append((kind, torch.ones(n, device=dev), None))
        else:
            bufs.append((kind, torch.ones(n, device=dev), torch.empty(world, n, device=dev)))

    def replay(only=None):
        for kind, x, out in bufs:
            if only and kind != only:
                continue
            if kind == "all_reduce":
                dist.all_reduce(x)
            elif backend == "nccl":
                dist.all_gather_into_tensor(out, x)
            else:
                dist.all_gather(list(out.unbind(0)), x)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t_all = timed(replay)
    t_ar = timed(lambda: replay("all_reduce"))
    t_ag = timed(lambda: replay("all_gather"))
    ar_bytes = 4 * sum(n for k, n in seq if k == "all_reduce")
    ag_bytes = 4 * sum(n for k, n in seq if k == "all_gather")
    return {"backend": backend, "collectives_per_step": len(seq),
            "sequence": [[k, n] for k, n in seq],
            "replay_ms": round(t_all * 1e3, 4),
            "all_reduce": {"calls": sum(1 for k, _ in seq if k == "all_reduce"), "bytes": ar_bytes,
                           "ms": round(t_ar * 1e3, 4),
                           "bus_GBps": round(2 * (world - 1) / world * ar_bytes / t_ar / 1e9, 2) if t_ar else None},
            "all_gather": {"calls": sum(1 for k, _ in seq if k == "all_gather"), "bytes_per_rank": ag_bytes,
                           "ms": round(t_ag * 1e3, 4),
                           "bus_GBps": round((world - 1) * ag_bytes / t_ag / 1e9, 2) if t_ag else None}}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--P", type=int, default=P_M1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--chunks", type=int, default=4, help="gradient exchange chunks (N > 1)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (r3dg_set_options, include/r3dg_hip.h) for A/B runs, e.g. test_no_cull=1")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; R3DG_DIST_BACKEND=gloo rehearses the multi-rank path on a single GPU
    backend = os.environ.get("R3DG_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    if world > 1:
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import relightable3dgaussian_amd as r3
    from relightable3dgaussian_amd import synthetic

    _C = r3._C
    if args.opt:
        _C.set_options({k: int(v) for k, v in (o.split("=", 1) for o in args.opt)})
    from relightable3dgaussian_amd import view_parallel

    cam = view_parallel.rank_camera(synthetic.m1_camera(W_M1, H_M1), rank, world)
    scene = synthetic.m1_scene(P=args.P, S=S_M1, seed=0, cam=synthetic.m1_camera(W_M1, H_M1))
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=dev)  # noqa: E731
    means3D, feats, opac = t(scene.means3D), t(scene.features), t(scene.opacity)
    scales, rots, sh = t(scene.scales), t(scene.rotations), t(scene.sh)
    empty = torch.empty(0, device=dev)
    bg = t([1.0, 1.0, 1.0])
    view, view_inv, proj, proj_inv, campos = t(cam.view), t(cam.view_inv), t(cam.proj), t(cam.proj_inv), t(cam.campos)
    H, W = cam.height, cam.width
    rng = np.random.default_rng(1)
    g_color = t(rng.normal(size=(3, H, W)) * 1e-3)
    g_opac = t(rng.normal(size=(H, W)) * 1e-3)
    g_depth = t(rng.normal(size=(H, W)) * 1e-3)
    g_feat = t(rng.normal(size=(S_M1, H, W)) * 1e-3)

    def step(exchange=True):
        out = _C.rasterize_gaussians(bg, 0.0, 0.0, means3D, feats, empty, opac, scales, rots, 1.0, empty, view,
                                     view_inv, proj, proj_inv, cam.tanfovx, cam.tanfovy, cam.cx, cam.cy, H, W, sh, 3,
                                     campos, False, True, None, None, None, None, False)
        L, radii, geom, binning, img = out[0], out[10], out[11], out[12], out[13]
        if world > 1 and exchange:
            # per-Gaussian gradients all-reduced chunk by chunk, overlapped with the gather phase
            view_parallel.backward_all_reduce(
                _C, (bg, means3D, feats, radii, empty, scales, rots, 1.0, empty, view, proj, cam.tanfovx,
                     cam.tanfovy, g_color, g_opac, g_depth, g_feat, sh, 3, campos, geom, L, binning, img, True,
                     False, H, W, False, False), n_chunks=args.chunks)
        else:
            _C.rasterize_gaussians_backward(bg, means3D, feats, radii, empty, scales, rots, 1.0, empty, view,
                                            proj, cam.tanfovx, cam.tanfovy, g_color, g_opac, g_depth, g_feat,
                                            sh, 3, campos, geom, L, binning, img, True, False)
        return L

    def run(fn, k):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            out = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0, out

    for _ in range(args.warmup):
        L = step()
    elapsed, L = run(step, args.steps)
    exchange = None
    if world > 1:
        # outside the timed region: the same steps without the gradient exchange (each rank's
        # compute alone, max over ranks) and the two collectives alone at this size
        t_comp, _ = run(lambda: step(exchange=False), args.steps)
        tc = torch.tensor([t_comp], dtype=torch.float64, device=dev)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        t_comp = float(tc.item())
        exchange = comm_probe(list(view_parallel.LAST_COLLECTIVES["sequence"]), dev, world, backend)
    # per-kernel device times: K more steps with HIP events inside the profiled launches (kept out
    # of the timed region above)
    _C.profile_enable(args.steps + 1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    prof = {k: _C.profile_read(i) for i, k in enumerate(["render_fwd", "render_bwd", "gather_bwd", "sort",
                                                          "preprocess", "row_sum"])}
    _C.profile_enable(0)
    if world > 1:
        te = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = float(te.item())
    if rank != 0:
        dist.destroy_process_group()
        return

    ms_step = elapsed / args.steps * 1e3
    npix = H * W
    value = world * npix * args.steps / elapsed / 1e6
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    bf, bb = algorithmic_bytes(L, npix, tiles, S_M1)
    # per-step device time of each stage
    avg = {k: v[1] / args.steps for k, v in prof.items()}
    launch = {k: (v[1] / v[0] if v[0] else 0.0) for k, v in prof.items()}
    # renderCUDA fwd + bwd: the backward blend AND its per-instance reduction's second stage (the
    # default atomic flush: the sums are zeroed inside render_fwd, the slot is empty; rows reduction:
    # row_sum_kernel, which sums the partial rows the reference accumulates with atomics,
    # backward.cu:552-611)
    reduce_mode = "rows" if _C.get_options()["bwd_reduce"] == 1 else "atomic"
    t_kern = (launch["render_fwd"] + launch["render_bwd"] + launch["row_sum"]) / 1e3
    achieved = (bf + bb) / t_kern / 1e9
    traffic = None
    tr = load_traffic()
    if tr and tr.get("config") == f"M1 P={args.P}":
        traffic = tr.get("render_fwd_bytes", 0) + tr.get("render_bwd_bytes", 0) + tr.get("row_sum_bytes", 0)
    valu = valu_roofline(load_valu(args.P), launch)
    res = {
        "metric": "Mpix/s fwd+bwd, 1M Gaussians @1920x1080; views/s at 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md §8d M1 generator, seed 0; no datasets offline)",
        "config": {"workload": "M1: rasterize_gaussians + rasterize_gaussians_backward, 1M Gaussians, 1920x1080, "
                               "S=11 features, SH degree 3, default shaders, pseudo normal",
                   "gaussians": args.P, "width": W, "height": H, "features": S_M1, "num_rendered": int(L),
                   "parallelism": f"view-parallel dp{world} (per Gaussian: RCCL all-reduce of the 22 packed dense floats + "
                                  f"all-gather of the 3-float SH colour gradient, SH sum rebuilt per rank; "
                                  f"{args.chunks} chunks overlapped with the gather phase, 2 collectives per chunk "
                                  f"+ 1 camera-centre all-gather per step)"},
        "views_per_s": round(world * args.steps / elapsed, 3),
        # priced against HBM (north_star: no dense contraction, the blend's bytes over 8 TB/s); which
        # resource binds is derived from the measured fractions (DESIGN.md §4 "Can 0.40 be reached")
        "roofline": {"bound": "hbm", "priced_against": "hbm",
                     "bound_note": "`bound` names the peak the kernel is priced against (the contract's hbm|mfma); "
                                   "the limiter measured from the hbm and valu fractions is `binding`",
                     "binding": binding(achieved / HBM_PEAK_GBS, valu), "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "renderCUDA fwd + bwd: render_fwd_glds_kernel + render_bwd_glds_kernel + the reduction's "
                               "second stage (the sums memset with the default atomic flush; row_sum_kernel with "
                               "R3DG_BWD_REDUCE=rows)",
                     "algorithmic_bytes": bf + bb, "extra_bytes": fused_sort_bytes(L),
                     "extra_bytes_note": "fused per-tile depth sort in the forward (12 B per instance), not in frac",
                     "kernel_ms": round(t_kern * 1e3, 4), "valu": valu},
        "kernel_ms": {("bwd_reduce_" + reduce_mode if k == "row_sum" else k): round(v, 4) for k, v in avg.items()
                      if prof[k][0]},
        "bwd_reduce": {"mode": reduce_mode,
                       "stage": ("the per-Gaussian sums are zeroed inside render_fwd (the training forward "
                                 "prepares them) and summed by render_bwd's atomic flush: no separate launch"
                                 if not prof["row_sum"][0] else "hipMemsetAsync of the per-Gaussian sums + the atomic "
                                 "flush inside render_bwd")
                       if reduce_mode == "atomic" else "row_sum_kernel over the partial rows"},
    }
    if exchange is not None:
        res["collectives_per_step"] = exchange["collectives_per_step"]
        ms_comp = t_comp / args.steps * 1e3
        exchange["compute_only_ms_per_step"] = round(ms_comp, 4)
        exchange["exposed_exchange_ms_per_step"] = round(ms_step - ms_comp, 4)
        exchange["exposed_frac_of_view"] = round((ms_step - ms_comp) / ms_comp, 4)
        res["exchange"] = exchange
    if world == 1:
        res["bvh_visibility"] = bvh_visibility(means3D, scales, rots, dev)
    if not args.no_cpu_baseline and world == 1:
        res["cpu_baseline"] = cpu_baseline(scene)
        res["brdf_cpu_baseline"] = brdf_c1(dev)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
