"""Golden vectors for the BVH leaf boxes from the REFERENCE's own RayTracer code (CPU container).

Runs the reference's `bvh.RayTracer.__init__` (bvh/__init__.py:28-61) on CPU on seeded inputs and
stores what it hands to the CUDA `_C.create_bvh`: the initial `nodes` table and the `aabbs`
table with the 8-corner leaf boxes of every Gaussian (rows P-1..2P-2), computed by the
reference's torch code with its `build_rotation` (utils/general_utils.py:82-103).

  bvh.npz  means3D, scales, rotations (inputs), nodes_init [2P-1,5], aabbs_init [2P-1,6]

How the reference is run: `torch.utils.cpp_extension.load` is replaced by a stub that returns an
object whose `create_bvh` records its arguments (the CUDA build cannot run here: no nvcc / GPU),
and make_golden.CpuMode rewrites the reference's device='cuda' allocations to CPU. The tree build
and the traces themselves have no CPU form in the reference; see oracle/r3dg_bvh.c for how those
are pinned.

Usage:  python tests/golden/make_golden_bvh.py  [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import CpuMode  # noqa: E402


class _RecordingC:
    def __init__(self):
        self.calls = []

    def create_bvh(self, means3D, scales, rotations, nodes, aabbs):
        self.calls.append((nodes.clone(), aabbs.clone()))
        return nodes, aabbs, torch.zeros(means3D.shape[0], dtype=torch.int64)


def load_bvh(ref: str):
    sys.path.insert(0, ref)
    import torch.utils.cpp_extension as cpp

    rec = _RecordingC()
    cpp.load = lambda *a, **k: rec  # the reference JIT-compiles its CUDA sources here
    spec = importlib.util.spec_from_file_location("bvh", os.path.join(ref, "bvh", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, rec


def scene(P: int, seed: int):
    rng = np.random.default_rng(seed)
    means = rng.uniform(-1.0, 1.0, (P, 3))
    scales = np.exp(rng.uniform(np.log(0.003), np.log(0.05), (P, 3)))
    rots = rng.normal(size=(P, 4))
    rots /= np.linalg.norm(rots, axis=1, keepdims=True)  # get_rotation is normalised
    rots *= rng.uniform(0.5, 2.0, (P, 1))  # ... build_rotation re-normalises: exercise it
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    return f(means), f(scales), f(rots)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    mod, rec = load_bvh(args.reference)
    P = 1024
    means, scales, rots = scene(P, 7)
    with CpuMode():
        mod.RayTracer(torch.from_numpy(means), torch.from_numpy(scales), torch.from_numpy(rots))
    nodes, aabbs = rec.calls[-1]
    np.savez_compressed(os.path.join(HERE, "bvh.npz"), means3D=means, scales=scales, rotations=rots,
                        nodes_init=nodes.numpy().astype(np.int32), aabbs_init=aabbs.numpy().astype(np.float32))
    print("wrote bvh.npz", nodes.shape, aabbs.shape)


if __name__ == "__main__":
    main()
