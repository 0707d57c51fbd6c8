"""MI355X-native relightable Gaussian-splat rasterizer (drop-in for r3dg_rasterization._C).

`relightable3dgaussian_amd._C` is the pybind module built from csrc/torch_ext.cpp on top of
lib/libr3dg_hip.so (HIP kernels for gfx950 + the C ABI in include/r3dg_hip.h). There is no
CPU fallback: importing `_C` raises if the extension has not been built, and every operator
requires GPU tensors.

`install_alias()` registers this package as `r3dg_rasterization` so the reference's
`from r3dg_rasterization import _C` (gaussian_renderer/r3dg_rasterization.py:7-8,
scene/gaussian_model.py:18) resolves here, and `relightable3dgaussian_amd.bvh` as the reference's
`bvh` package (`from bvh import RayTracer`, scene/gaussian_model.py:16).
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys

import torch  # noqa: F401  (loads libtorch / the HIP runtime before our libraries)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.environ.get("R3DG_LIB_DIR") or os.path.join(_PKG, "lib")  # override: experiment builds
HIP_LIB = os.path.join(LIB_DIR, "libr3dg_hip.so")
EXT_LIB = os.path.join(LIB_DIR, "_C.so")


def _load_ext():
    if not os.path.exists(EXT_LIB) or not os.path.exists(HIP_LIB):
        raise ImportError(
            "relightable3dgaussian_amd: native extension not built (expected %s and %s); run "
            "`python relightable3dgaussian_amd/build.py` or __graft_entry__.build()" % (HIP_LIB, EXT_LIB))
    loader = importlib.machinery.ExtensionFileLoader("relightable3dgaussian_amd._C", EXT_LIB)
    spec = importlib.util.spec_from_file_location("relightable3dgaussian_amd._C", EXT_LIB, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules["relightable3dgaussian_amd._C"] = mod
    return mod


_C = _load_ext()


def install_alias() -> None:
    """Make `import r3dg_rasterization` / `from r3dg_rasterization import _C` resolve here."""
    from . import r3dg_rasterization as wrapper

    sys.modules.setdefault("r3dg_rasterization", wrapper)
    sys.modules.setdefault("r3dg_rasterization._C", _C)
    # the reference's BVH tracer package (bvh/__init__.py) and its extension bvh_tracing._C
    from .bvh import install_bvh_alias

    install_bvh_alias()


__all__ = ["_C", "install_alias", "HIP_LIB", "EXT_LIB"]
