"""Timings for DESIGN §6 (view-parallel exchange cost model) and the C3 optimizer step, 1 GPU.

  * M1 backward per-Gaussian phase (row-sum + gather) in one chunk vs the 4 chunks the
    view-parallel exchange overlaps with (_C.rasterize_gaussians_backward_chunked);
  * the "views" SH exchange kernels at M1 for N = 8 views: r3dg_sh_color_grads per view and
    r3dg_sh_grad_from_views over the 8 gathered colour gradients;
  * C3's trainer step at P = 250k (14-group NeILF model): _C.adam_step alone and st.step.
Writes one JSON object (stdout and --out). Usage: python tools/bench_views.py [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20, warm=3):
    import torch

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    import relightable3dgaussian_amd as r3
    from relightable3dgaussian_amd import synthetic, trainer
    from tests._helpers import hip_forward, tt, upstream_grads

    _C = r3._C
    res = {}
    cam = synthetic.m1_camera()
    scene = synthetic.m1_scene(P=1_000_000, S=11, seed=0, cam=cam)
    P = scene.P
    h = hip_forward(_C, scene, cam, S=11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=3)
    ar = h["_args"]
    args = (tt(h["_bg"]), ar["means3D"], ar["features"], h["radii"], ar["colors"], ar["scales"], ar["rotations"], 1.0,
            ar["cov3D"], tt(cam.view), tt(cam.proj), cam.tanfovx, cam.tanfovy, tt(dc), tt(do), tt(dd), tt(df),
            ar["sh"], 3, tt(cam.campos), h["geom"], h["num_rendered"], h["binning"], h["image"], True, False,
            cam.height, cam.width, False, False)
    res["m1_backward_1chunk_ms"] = timed(lambda: _C.rasterize_gaussians_backward_chunked(*args, 1, None))
    res["m1_backward_4chunks_ms"] = timed(lambda: _C.rasterize_gaussians_backward_chunked(*args, 4, None))
    grads = _C.rasterize_gaussians_backward_chunked(*args, 1, None)
    dcol = grads[1].contiguous()
    res["sh_color_grads_ms"] = timed(lambda: _C.sh_color_grads(h["geom"], P, dcol, 0, P))
    d = _C.sh_color_grads(h["geom"], P, dcol, 0, P)
    d_all = torch.stack([d] * 8).contiguous()
    cams = tt(np.stack([np.asarray(cam.campos, np.float32) + np.float32(0.01 * k) for k in range(8)]))
    out = torch.empty((P, 16, 3), device="cuda")
    res["sh_grad_from_views_n8_ms"] = timed(lambda: _C.sh_grad_from_views(ar["means3D"], cams, d_all, 3, 0, out))
    # bytes per Gaussian on the wire per GPU at N = 8 (ring): all-reduce of 22 floats + all-gather of 3
    res["views_exchange_bytes_per_gaussian_n8"] = 2 * 7 / 8 * 88 + 7 * 12
    del h, grads

    # C3 optimizer step
    Pc = 250_000
    rng = np.random.default_rng(0)
    shapes = dict(trainer.BASE_GROUPS + trainer.PBR_GROUPS)
    t = {n: torch.from_numpy(rng.normal(size=(Pc,) + s).astype(np.float32)).cuda() for n, s in shapes.items()}
    st = trainer.GaussianTrainState.from_tensors(t)
    st.training_setup(types.SimpleNamespace(
        percent_dense=0.01, position_lr_init=0.00016, position_lr_final=0.0000016, position_lr_delay_mult=0.01,
        position_lr_max_steps=30000, normal_lr=0.01, rotation_lr=0.001, scaling_lr=0.005, opacity_lr=0.05,
        sh_lr=0.0025, base_color_lr=0.01, roughness_lr=0.01, metallic_lr=0.01, light_lr=0.002, light_rest_lr=-1.0,
        visibility_lr=0.0025, visibility_rest_lr=-1.0))
    n = st.total()
    st.grad[:n] = torch.randn(n, device="cuda") * 1e-3

    def adam_only():
        st.step_count += 1
        _C.adam_step(st.P, st.widths(), st.roles(), st.param, st.grad[:n], st.exp_avg[:n], st.exp_avg_sq[:n], 0, n,
                     list(st.lrs), 0.9, 0.999, 1e-15, st.step_count)

    res["c3_floats"] = n
    res["c3_adam_kernel_ms"] = timed(adam_only, 50)
    res["c3_adam_tbps"] = 28.0 * n / (res["c3_adam_kernel_ms"] * 1e-3) / 1e12
    res["c3_st_step_ms"] = timed(st.step, 50)
    res["c3_st_step_zero_grad_ms"] = timed(lambda: st.step(zero_grad=True), 50)
    res = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
