"""Timing of BASELINE.json's other GPU configs on 1 GPU (SURVEY.md §8d stand-ins; the bench line is
M1 = configs[3]-style 1080p fwd+bwd). Synthetic scenes, no checkpoints exist offline:

  C2  lego stand-in: ball_scene P=300k, S=21, 800x800, orbit camera (radius 4.0311, fov 0.6911,
      elevation 30 deg), white background: rasterize_gaussians + render_equation_forward_complex
      (eval BRDF, Ns=24) -- "forward raster + BRDF";
  C3  hotdog training step stand-in: ball_scene seed 2, P=250k, S=11, same camera:
      rasterize fwd + bwd, render_equation_forward (training, random rotation) + backward, and
      the device Adam step over the 14-group NeILF model (trainer.GaussianTrainState.step);
  C4  truck stand-in: M1 generator with P=2M, 1920x1080, rasterize fwd + bwd.
Median of --iters timed iterations after warmup, HIP events on the current stream.

Usage: python tools/bench_configs.py [--iters 10] [--out profiles/r01_configs.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    import relightable3dgaussian_amd as r3
    from relightable3dgaussian_amd import synthetic, trainer

    _C = r3._C
    dev = torch.device("cuda", 0)
    T = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float32, device=dev)  # noqa: E731
    empty = torch.empty(0, device=dev)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    def raster(scene, cam, bg):
        g = dict(means3D=T(scene.means3D), feats=T(scene.features), opac=T(scene.opacity), scales=T(scene.scales),
                 rots=T(scene.rotations), sh=T(scene.sh))
        c = dict(view=T(cam.view), view_inv=T(cam.view_inv), proj=T(cam.proj), proj_inv=T(cam.proj_inv),
                 campos=T(cam.campos))
        bgt = T(bg)

        def fwd():
            return _C.rasterize_gaussians(bgt, 0.0, 0.0, g["means3D"], g["feats"], empty, g["opac"], g["scales"],
                                          g["rots"], 1.0, empty, c["view"], c["view_inv"], c["proj"], c["proj_inv"],
                                          cam.tanfovx, cam.tanfovy, cam.cx, cam.cy, cam.height, cam.width, g["sh"], 3,
                                          c["campos"], False, True, None, None, None, None, False)

        S = scene.features.shape[1]
        rng = np.random.default_rng(1)
        H, W = cam.height, cam.width
        gr = [T(rng.normal(size=s) * 1e-3) for s in [(3, H, W), (H, W), (H, W), (S, H, W)]]

        def fwd_bwd():
            out = fwd()
            return _C.rasterize_gaussians_backward(bgt, g["means3D"], g["feats"], out[10], empty, g["scales"],
                                                   g["rots"], 1.0, empty, c["view"], c["proj"], cam.tanfovx,
                                                   cam.tanfovy, *gr, g["sh"], 3, c["campos"], out[11], out[0],
                                                   out[12], out[13], True, False)
        return fwd, fwd_bwd

    res = {}
    lego_cam = synthetic.orbit_camera(0.0, 30.0, 4.0311, 0.6911112, 800, 800)
    # C2: forward raster + eval BRDF
    sc = synthetic.ball_scene(300_000, S=21, seed=0)
    fwd, _ = raster(sc, lego_cam, [1.0, 1.0, 1.0])
    b = {k: T(v) for k, v in synthetic.brdf_inputs(300_000, seed=0).items()}
    bargs = [b["base"], b["rough"], b["metal"], b["normals"], b["viewdirs"], b["incidents"], b["env"], b["visibility"]]
    L = fwd()[0]
    t_r = timed(fwd)
    t_b = timed(lambda: _C.render_equation_forward_complex(*bargs, 24))
    res["C2"] = {"workload": "ball P=300k S=21 800x800 fwd raster + BRDF complex fwd (Ns=24)", "num_rendered": int(L),
                 "raster_fwd_ms": round(t_r, 4), "brdf_complex_fwd_ms": round(t_b, 4),
                 "total_ms": round(t_r + t_b, 4), "views_per_s": round(1e3 / (t_r + t_b), 1)}
    # C3: training step (raster fwd+bwd, training BRDF fwd+bwd, Adam over the NeILF model)
    P3 = 250_000
    sc = synthetic.ball_scene(P3, S=11, seed=2)
    _, fwd_bwd = raster(sc, lego_cam, [1.0, 1.0, 1.0])
    b = {k: T(v) for k, v in synthetic.brdf_inputs(P3, seed=2).items()}
    bargs = [b["base"], b["rough"], b["metal"], b["normals"], b["viewdirs"], b["incidents"], b["env"], b["visibility"]]
    ones = torch.ones(P3, 3, device=dev)
    rng = np.random.default_rng(3)
    shapes = dict(trainer.BASE_GROUPS + trainer.PBR_GROUPS)
    st = trainer.GaussianTrainState.from_tensors(
        {n: T(rng.normal(size=(P3,) + s) * 0.1) for n, s in shapes.items()})
    st.training_setup(types.SimpleNamespace(
        percent_dense=0.01, position_lr_init=0.00016, position_lr_final=0.0000016, position_lr_delay_mult=0.01,
        position_lr_max_steps=30000, normal_lr=0.01, rotation_lr=0.001, scaling_lr=0.005, opacity_lr=0.05,
        sh_lr=0.0025, base_color_lr=0.01, roughness_lr=0.01, metallic_lr=0.01, light_lr=0.002, light_rest_lr=-1.0,
        visibility_lr=0.0025, visibility_rest_lr=-1.0))

    def brdf_step():
        pbr, dirs, dl = _C.render_equation_forward(*bargs, 24, True, False)
        _C.render_equation_backward(*bargs, 24, dirs, ones, ones, False)

    t_rfb = timed(fwd_bwd)
    t_bfb = timed(brdf_step)
    t_adam = timed(st.step)
    tot = t_rfb + t_bfb + t_adam
    res["C3"] = {"workload": "ball seed 2 P=250k S=11 800x800: raster fwd+bwd + BRDF training fwd+bwd + Adam (131 "
                             "floats/Gaussian)", "raster_fwd_bwd_ms": round(t_rfb, 4),
                 "brdf_fwd_bwd_ms": round(t_bfb, 4), "adam_ms": round(t_adam, 4), "total_ms": round(tot, 4),
                 "steps_per_s": round(1e3 / tot, 1)}
    # C4: truck stand-in, 2M Gaussians at 1080p
    cam4 = synthetic.m1_camera(1920, 1080)
    sc = synthetic.m1_scene(P=2_000_000, S=11, seed=0, cam=cam4)
    fwd4, fwd_bwd4 = raster(sc, cam4, [1.0, 1.0, 1.0])
    L4 = fwd4()[0]
    t4 = timed(fwd_bwd4)
    res["C4"] = {"workload": "M1 generator P=2M S=11 1920x1080 fwd+bwd", "num_rendered": int(L4),
                 "ms": round(t4, 4), "Mpix_per_s": round(1920 * 1080 / t4 / 1e3, 1)}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
