"""BVH visibility tracer: drop-in for the reference's `bvh` package (bvh/__init__.py).

The reference builds a linear BVH over the Gaussians' 3-sigma boxes and traces visibility rays
through it (gaussian_renderer/neilf.py:323-348 `lambda_visibility`, scene/gaussian_model.py:430-466
`finetune_visibility`, relighting.py:74). Here:

  * `RayTracer(means3D, scales, rotations)` -- same constructor, same `tree` / `aabb` / `morton`
    attributes (the reference's layouts); the leaf boxes come from one HIP launch
    (`_C.bvh_leaf_aabbs`) instead of ~40 torch ops, the tree from `_C.create_bvh`.
  * `trace_visibility(rays_o, rays_d, means3D, symm_inv, opacity, normals)` -- same dict
    {"visibility": [..., 1], "contribute": [..., 1]} via `_C.trace_bvh_opacity`.
  * `_C` here is the package's extension, which carries the reference's `bvh_tracing._C` names
    (`create_bvh`, `trace_bvh`, `trace_bvh_opacity`); `install_bvh_alias()` registers this module as
    `bvh` and the extension as `bvh_tracing._C`.

No CPU path: the extension rejects CPU tensors (the reference's module is CUDA-only too).
"""
from __future__ import annotations

import sys
import types

import torch

from . import _C


class RayTracer:
    """bvh/__init__.py:28-69."""

    def __init__(self, means3D, scales, rotations):
        P = means3D.shape[0]
        dev = means3D.device
        nodes = torch.empty((2 * P - 1, 5), dtype=torch.int32, device=dev)  # every field is written
        aabbs = torch.empty((2 * P - 1, 6), dtype=torch.float32, device=dev)
        aabbs[P - 1:] = _C.bvh_leaf_aabbs(means3D.float(), scales.float(), rotations.float())
        self.tree, self.aabb, self.morton = _C.create_bvh(means3D, scales, rotations, nodes, aabbs)

    @torch.no_grad()
    def trace_visibility(self, rays_o, rays_d, means3D, symm_inv, opacity, normals):
        contrib, opa = _C.trace_bvh_opacity(self.tree, self.aabb, rays_o, rays_d, means3D, symm_inv, opacity,
                                            normals)
        return {"visibility": opa.unsqueeze(-1), "contribute": contrib.unsqueeze(-1)}


def install_bvh_alias() -> None:
    """Make `from bvh import RayTracer` and `from bvh_tracing import _C` resolve here."""
    sys.modules.setdefault("bvh", sys.modules[__name__])
    pkg = sys.modules.get("bvh_tracing")
    if pkg is None:
        pkg = types.ModuleType("bvh_tracing")
        pkg._C = _C
        sys.modules["bvh_tracing"] = pkg
    sys.modules.setdefault("bvh_tracing._C", _C)


__all__ = ["RayTracer", "install_bvh_alias"]
