"""Per-kernel device times (the library's profiled launches, as bench.py) of the C3 raster step
(tools/bench_configs.py's C3 scene: ball_scene seed 2, P = 250k, S = 11, 800 x 800) and of C4.
Usage: python tools/bench_c3_kernels.py [--steps 20]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import relightable3dgaussian_amd as r3
    from relightable3dgaussian_amd import synthetic

    _C = r3._C
    dev = torch.device("cuda", 0)
    T = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float32, device=dev)  # noqa: E731
    empty = torch.empty(0, device=dev)
    names = ["render_fwd", "render_bwd", "gather_bwd", "sort", "preprocess", "row_sum"]
    res = {}
    for tag, sc, cam in [("C3", synthetic.ball_scene(250_000, S=11, seed=2),
                          synthetic.orbit_camera(0.0, 30.0, 4.0311, 0.6911112, 800, 800))]:
        bg = T([1.0, 1.0, 1.0])
        g = [T(sc.means3D), T(sc.features), T(sc.opacity), T(sc.scales), T(sc.rotations), T(sc.sh)]
        c = [T(cam.view), T(cam.view_inv), T(cam.proj), T(cam.proj_inv), T(cam.campos)]
        H, W, S = cam.height, cam.width, sc.features.shape[1]
        rng = np.random.default_rng(1)
        gr = [T(rng.normal(size=s) * 1e-3) for s in [(3, H, W), (H, W), (H, W), (S, H, W)]]

        def step():
            out = _C.rasterize_gaussians(bg, 0.0, 0.0, g[0], g[1], empty, g[2], g[3], g[4], 1.0, empty, c[0], c[1],
                                         c[2], c[3], cam.tanfovx, cam.tanfovy, cam.cx, cam.cy, H, W, g[5], 3, c[4],
                                         False, True, None, None, None, None, False)
            _C.rasterize_gaussians_backward(bg, g[0], g[1], out[10], empty, g[3], g[4], 1.0, empty, c[0], c[2],
                                            cam.tanfovx, cam.tanfovy, *gr, g[5], 3, c[4], out[11], out[0], out[12],
                                            out[13], True, False)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            step()
        e1.record()
        e1.synchronize()
        _C.profile_enable(a.steps + 1)
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        prof = {k: round(_C.profile_read(i)[1] / a.steps, 4) for i, k in enumerate(names)}
        _C.profile_enable(0)
        res[tag] = {"ms_per_step": round(e0.elapsed_time(e1) / a.steps, 4), "kernel_ms": prof}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
