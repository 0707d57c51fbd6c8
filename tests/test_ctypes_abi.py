"""The C ABI through raw ctypes, exactly as INTEGRATION.md §2 shows a maintainer would bind it
(no torch extension in the call path): include/r3dg_hip.h entry points on device pointers and the
caller's HIP stream, checked against the oracle and the torch binding."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle
from relightable3dgaussian_amd import synthetic

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def abi():
    import torch  # noqa: F401  (loads the HIP runtime the library shares)

    import relightable3dgaussian_amd as r3

    lib = ctypes.CDLL(os.path.join(r3.LIB_DIR, "libr3dg_hip.so"))
    lib.r3dg_last_error.restype = ctypes.c_char_p
    return lib


def _stream():
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def test_mark_visible_raw_ctypes(abi):
    """r3dg_mark_visible <- rasterize_points.cu:277-295 (markVisible), INTEGRATION.md's binding."""
    import torch

    scene, cam = synthetic.small_scene(P=4000, seed=31)
    m = scene.means3D.copy()
    m[::4, 2] *= -1  # a quarter behind the camera
    means3D = torch.tensor(m, device="cuda")
    view = torch.tensor(cam.view, device="cuda")
    proj = torch.tensor(cam.proj, device="cuda")
    out = torch.empty(means3D.shape[0], dtype=torch.bool, device="cuda")
    rc = abi.r3dg_mark_visible(ctypes.c_int(means3D.shape[0]), ctypes.c_void_p(means3D.data_ptr()),
                               ctypes.c_void_p(view.data_ptr()), ctypes.c_void_p(proj.data_ptr()),
                               ctypes.c_void_p(out.data_ptr()), _stream())
    assert rc == 0, abi.r3dg_last_error()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.mark_visible(m, cam.view))
    # errors come back as codes with text, not crashes: P < 0 is refused or a no-op, never a launch
    assert abi.r3dg_mark_visible(ctypes.c_int(0), None, None, None, None, _stream()) == 0


def test_trace_bvh_opacity_raw_ctypes(abi):
    """r3dg_bvh_trace_opacity <- bvh/src/bvh.cu:87-117 through ctypes with a torch-backed
    r3dg_alloc_fn callback, bit-identical to the torch binding's result."""
    import torch

    import relightable3dgaussian_amd as r3
    from tests.test_bvh import hip_build, rays_from, scene, tt

    sc = scene(3000, seed=17, spread=0.5)
    _, nodes, aabbs, _ = hip_build(r3._C, sc)
    o, d = rays_from(sc, 2000, seed=5)
    rays_o, rays_d = tt(o), tt(d)
    means3D, cov_inv = tt(sc["means"]), tt(sc["cov_inv"])
    opacity, normals = tt(sc["opacity"]), tt(sc["normals"])

    ALLOC = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
    keep = []

    @ALLOC
    def torch_alloc(ctx, nbytes):
        t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda")
        keep.append(t)
        return t.data_ptr()

    R, P = rays_o.numel() // 3, means3D.shape[0]
    contrib = torch.zeros(rays_o.shape[:-1], dtype=torch.int32, device="cuda")
    vis = torch.ones(rays_o.shape[:-1], device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = abi.r3dg_bvh_trace_opacity(ctypes.c_int(R), ctypes.c_int(P), p(nodes), p(aabbs), p(rays_o), p(rays_d),
                                    p(means3D), p(cov_inv), p(opacity), p(normals), p(contrib), p(vis), torch_alloc,
                                    None, _stream())
    assert rc == 0, abi.r3dg_last_error()
    c_ref, v_ref = r3._C.trace_bvh_opacity(nodes, aabbs, rays_o, rays_d, means3D, cov_inv, opacity, normals)
    torch.cuda.synchronize()
    assert torch.equal(contrib.reshape(-1), c_ref.reshape(-1))
    assert torch.equal(vis.reshape(-1), v_ref.reshape(-1))
    assert int(contrib.sum()) > 0
