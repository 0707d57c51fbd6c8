"""BVH visibility tracer timing on one MI355X.

Workloads (the reference's call sites, synthetic scenes of the M1 generator's size class):
  build   RayTracer(means3D, scales, rotations) at P Gaussians (bvh/__init__.py:28-61)
  trace   trace_visibility with R rays from Gaussian centres, directions flipped into the normal's
          hemisphere (finetune_visibility: R = P, gaussian_model.py:446-465; lambda_visibility:
          R = 10k, neilf.py:323-348)
Also times the reference's own torch formulation of the leaf boxes (the ~40 elementwise ops of
bvh/__init__.py:29-59, restated here with torch on the same GPU) beside the one-launch kernel,
and the C oracle's trace on a bounded ray sample as the CPU baseline (1 thread).

Scenes: "volume" (tests/test_bvh.py scene: 1M Gaussians filling a cube -- every ray is blocked
within a short distance, a worst case for traversal length) and "surface" (Gaussians on sphere
shells, flattened along their outward normals: the geometry the visibility term is meant for).

Usage: python tools/bench_bvh.py [--P 1000000] [--rays 1000000] [--iters 10] [--scene volume|surface]
                                 [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def torch_leaf_boxes(means3D, scales, rotations):
    """The reference's RayTracer.__init__ box math as torch ops (bvh/__init__.py:29-59)."""
    r = rotations
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=q.device)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    a, b, c = R[:, :, 0], R[:, :, 1], R[:, :, 2]
    sa, sb, sc = 3 * scales[:, 0], 3 * scales[:, 1], 3 * scales[:, 2]
    corners = [means3D + i * a * sa[:, None] + j * b * sb[:, None] + k * c * sc[:, None]
               for i in (1, -1) for j in (1, -1) for k in (1, -1)]
    lo, hi = corners[0], corners[0]
    for v in corners[1:]:
        lo, hi = torch.minimum(lo, v), torch.maximum(hi, v)
    return torch.cat([lo, hi], -1)


def surface_scene(P, seed=0):
    """Gaussians on the shells of 12 spheres, flattened along the outward normal (a surface-like
    scene: rays from the centres into the normal's hemisphere either escape or hit another shell)."""
    import oracle

    rng = np.random.default_rng(seed)
    centers = rng.uniform(-1.0, 1.0, (12, 3))
    radii = rng.uniform(0.15, 0.4, 12)
    k = rng.integers(0, 12, P)
    n = rng.normal(size=(P, 3))
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    means = centers[k] + radii[k, None] * n
    s = np.exp(rng.uniform(np.log(0.004), np.log(0.015), (P, 1)))
    scales = np.concatenate([s, s, 0.1 * s], axis=1)
    # quaternion (w, x, y, z) rotating +z onto n
    z = np.array([0.0, 0.0, 1.0])
    axis = np.cross(np.broadcast_to(z, n.shape), n)
    w = 1.0 + n[:, 2]
    q = np.concatenate([w[:, None], axis], axis=1)
    q[w < 1e-6] = [0.0, 1.0, 0.0, 0.0]
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    sc = dict(means=f(means), scales=f(scales), rots=f(q), opacity=f(rng.uniform(0.3, 0.95, P)), normals=f(n))
    sc["cov_inv"] = f(oracle.cov3d(1.0 / sc["scales"], sc["rots"]))
    return sc


def timed(fn, iters, stream=None):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cpu-rays", type=int, default=20000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--scene", choices=["volume", "surface"], default="volume")
    args = ap.parse_args()
    import oracle
    import relightable3dgaussian_amd as r3
    from relightable3dgaussian_amd.bvh import RayTracer
    from tests.test_bvh import rays_from, scene

    torch.cuda.set_device(0)
    sc = scene(args.P, seed=8, spread=1.0) if args.scene == "volume" else surface_scene(args.P, seed=8)
    dev = lambda a: torch.as_tensor(a, device="cuda")  # noqa: E731
    means, scales, rots = dev(sc["means"]), dev(sc["scales"]), dev(sc["rots"])
    cov, opac, normals = dev(sc["cov_inv"]), dev(sc["opacity"]), dev(sc["normals"])
    res = {"P": args.P, "rays": args.rays, "scene": args.scene, "device": torch.cuda.get_device_name(0)}
    res["leaf_boxes_kernel_ms"] = timed(lambda: r3._C.bvh_leaf_aabbs(means, scales, rots), args.iters)
    res["leaf_boxes_torch_ms"] = timed(lambda: torch_leaf_boxes(means, scales, rots), args.iters)
    res["build_ms"] = timed(lambda: RayTracer(means, scales, rots), args.iters)
    rt = RayTracer(means, scales, rots)
    for R, key in ((args.rays, "trace"), (10000, "trace_10k")):
        o, d = rays_from(sc, R, seed=2)
        o, d = dev(o), dev(d)
        ms = timed(lambda: rt.trace_visibility(o, d, means, cov, opac, normals), args.iters)
        out = rt.trace_visibility(o, d, means, cov, opac, normals)
        res[key + "_ms"] = ms
        res[key + "_Mrays_per_s"] = R / ms / 1e3
        res[key + "_mean_visibility"] = float(out["visibility"].mean())
        res[key + "_occluded_frac"] = float((out["visibility"] == 0).float().mean())
    o, d = rays_from(sc, args.cpu_rays, seed=2)
    nodes, aabbs = rt.tree.cpu().numpy(), rt.aabb.cpu().numpy()
    t0 = time.perf_counter()
    oracle.bvh_trace_opacity(nodes, aabbs, o, d, sc["means"], sc["cov_inv"], sc["opacity"], sc["normals"])
    cpu_s = time.perf_counter() - t0
    res["cpu_baseline"] = {"kind": "port", "cores": 1, "Mrays_per_s": args.cpu_rays / cpu_s / 1e6,
                           "sample": f"oracle/r3dg_bvh.c trace_opacity, {args.cpu_rays} rays over the same tree"}
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
