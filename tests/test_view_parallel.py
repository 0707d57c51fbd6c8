"""World-size-2 gloo test of the view-parallel step (relightable3dgaussian_amd/view_parallel.py):
each rank renders its own camera, backward runs per rank, and one all-reduce of the flat gradient
bucket must equal the sum of the per-view gradients computed serially. The per-view gradients
come from the CPU oracle standing in for the kernel (tests may use it; the GPU path is covered by
the -m gpu parity tests); what is under test is the exchange logic bench.py uses."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest


def _per_view_grads(rank, world):
    import torch

    import oracle
    from relightable3dgaussian_amd import synthetic, view_parallel

    base = synthetic.m1_camera(64, 48)
    scene = synthetic.m1_scene(P=1500, S=5, seed=7, cam=base)
    cam = view_parallel.rank_camera(base, rank, world, step_deg=4.0)
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh,
                                 scales=scene.scales, rotations=scene.rotations)
    rng = np.random.default_rng(100 + rank)
    H, W = cam.height, cam.width
    g = oracle.rasterize_backward(o, rng.normal(size=(3, H, W)).astype(np.float32),
                                  rng.normal(size=(H, W)).astype(np.float32),
                                  rng.normal(size=(H, W)).astype(np.float32),
                                  rng.normal(size=(5, H, W)).astype(np.float32))
    order = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dfeatures", "dL_dcov3D", "dL_dsh",
             "dL_dscales", "dL_drotations"]
    return tuple(torch.from_numpy(np.ascontiguousarray(g[k])) for k in order)


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from relightable3dgaussian_amd import view_parallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _per_view_grads(rank, world)
        summed = view_parallel.all_reduce_grads(mine)
        ref = [_per_view_grads(r, world) for r in range(world)]
        err = 0.0
        for name, idx in view_parallel.GRAD_FIELDS:
            exp = sum(r[idx] for r in ref)
            err = max(err, float((summed[name] - exp).abs().max()))
        q.put((rank, err, float(summed["means3D"].abs().sum())))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_view_parallel_all_reduce_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, p.exitcode
    res = sorted(q.get(timeout=10) for _ in range(2))
    for rank, err, mag in res:
        assert err <= 1e-5 * max(mag, 1.0), (rank, err)
    assert res[0][2] == res[1][2]  # both ranks hold the identical summed gradient


def test_rank_cameras_differ_and_flatten_roundtrip():
    import torch

    from relightable3dgaussian_amd import synthetic, view_parallel

    base = synthetic.m1_camera(64, 48)
    c0, c1 = (view_parallel.rank_camera(base, r, 2) for r in range(2))
    assert not np.allclose(c0.view, c1.view)
    assert view_parallel.rank_camera(base, 0, 1) is base
    P, M, S = 5, 16, 3
    grads = (torch.randn(P, 3), torch.randn(P, 3), torch.randn(P, 1), torch.randn(P, 3), torch.randn(P, S),
             torch.randn(P, 6), torch.randn(P, M, 3), torch.randn(P, 3), torch.randn(P, 4))
    flat = view_parallel.flatten_grads(grads)
    assert flat.numel() == P * (3 + 3 * M + 1 + 3 + 4 + S)
    back = view_parallel.unflatten_grads(flat, grads)
    for name, idx in view_parallel.GRAD_FIELDS:
        assert torch.equal(back[name], grads[idx])


def _per_view_sh_inputs(rank, world):
    """One view's backward tuple (oracle), its clamp-masked colour gradients and camera centre."""
    import torch

    import oracle
    from oracle import view_exchange
    from relightable3dgaussian_amd import synthetic, view_parallel

    base = synthetic.m1_camera(64, 48)
    scene = synthetic.m1_scene(P=1500, S=5, seed=7, cam=base)
    cam = view_parallel.rank_camera(base, rank, world, step_deg=4.0)
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh,
                                 scales=scene.scales, rotations=scene.rotations)
    grads = _per_view_grads(rank, world)
    drgb = view_exchange.sh_color_grads(grads[1].numpy(), o["clamped"])
    return scene, grads, torch.from_numpy(drgb), torch.from_numpy(np.asarray(cam.campos, np.float32))


def test_sh_rebuild_oracle_matches_per_view_sums():
    """oracle/view_exchange.py (the rank-1 SH rebuild) against the C oracle's own per-view dL_dsh
    (backward.cu:20-139 restated), summed over three views."""
    from oracle import view_exchange

    views = [_per_view_sh_inputs(r, 3) for r in range(3)]
    scene = views[0][0]
    ref = sum(v[1][6].numpy() for v in views)
    got = view_exchange.sh_grad_from_views(scene.means3D, np.stack([v[3].numpy() for v in views]),
                                           np.stack([v[2].numpy() for v in views]), 3, 16)
    scale = float(np.abs(ref).max())
    assert scale > 0
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * scale)


def _views_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from oracle import view_exchange
    from relightable3dgaussian_amd import view_parallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene, grads, drgb, campos = _per_view_sh_inputs(rank, world)

        def rebuild(means3D, cams, d_all, degree, M):
            return torch.from_numpy(view_exchange.sh_grad_from_views(np.asarray(means3D), cams.numpy(),
                                                                     d_all.numpy(), degree, M))

        out = view_parallel.exchange_grads_views(grads, drgb, campos, scene.means3D, 3, rebuild)
        ref = [_per_view_grads(r, world) for r in range(world)]
        err = {}
        for name, idx in view_parallel.GRAD_FIELDS:
            exp = sum(r[idx] for r in ref)
            err[name] = (float((out[name] - exp).abs().max()), float(exp.abs().max()))
        q.put((rank, err, float(out["sh"].abs().sum())))
    finally:
        dist.destroy_process_group()


def test_view_parallel_views_exchange_gloo_world2():
    """The default "views" exchange (dense fields all-reduced, per-view SH colour gradients
    all-gathered, SH sum rebuilt on every rank) equals the serial sum of the per-view gradients,
    SH block included, and both ranks hold the identical result."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_views_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, p.exitcode
    res = sorted(q.get(timeout=10) for _ in range(2))
    for rank, err, _ in res:
        for name, (e, mag) in err.items():
            assert e <= 1e-5 * max(mag, 1e-12), (rank, name, e, mag)
    assert res[0][2] == res[1][2]
