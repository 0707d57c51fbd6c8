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


def _raw_forward(lib, A, scene, cam, S, keep):
    """r3dg_rasterize_gaussians_ex through ctypes (rasterize_points.cu:39-181's contract): inputs and
    outputs as torch tensors, the three state buffers and the scratch from a torch-backed r3dg_alloc_fn
    whose ctx names the buffer."""
    import torch

    from tests._helpers import tt

    H, W = cam.height, cam.width
    P = scene.P
    ins = {k: tt(v) for k, v in dict(means3D=scene.means3D, features=np.ascontiguousarray(scene.features[:, :S]),
                                     opacity=scene.opacity, scales=scene.scales, rotations=scene.rotations,
                                     sh=scene.sh, bg=np.ones(3, np.float32), view=cam.view, view_inv=cam.view_inv,
                                     proj=cam.proj, proj_inv=cam.proj_inv, campos=cam.campos).items()}
    keep.append(ins)
    f = lambda *s: torch.empty(*s, device="cuda")  # noqa: E731
    outs = dict(color=f(H, W, 3), opacity=f(H, W, 1), depth=f(H, W, 1), stencil=f(H, W, 1), feature=f(H, W, S),
                shader_color=f(H, W, 3), normal=f(H, W, 3), surface_xyz=f(H, W, 3),
                radii=torch.empty(P, dtype=torch.int32, device="cuda"))
    bufs = {}

    @A.ALLOC
    def alloc(ctx, n):
        t = torch.empty(max(int(n), 256), dtype=torch.uint8, device="cuda")
        bufs[ctx] = t
        return t.data_ptr()

    keep.append(alloc)
    p = lambda t: t.data_ptr()  # noqa: E731
    s = A.new(A.RasterSettings, P=P, S=S, D=3, M=scene.sh.shape[1], W=W, H=H, tan_fovx=cam.tanfovx,
              tan_fovy=cam.tanfovy, cx=cam.cx, cy=cam.cy, scale_modifier=1.0, compute_pseudo_normal=1,
              bg=p(ins["bg"]), viewmatrix=p(ins["view"]), viewmatrix_inv=p(ins["view_inv"]),
              projmatrix=p(ins["proj"]), projmatrix_inv=p(ins["proj_inv"]), campos=p(ins["campos"]))
    g = A.Gaussians(means3D=p(ins["means3D"]), features=p(ins["features"]), opacity=p(ins["opacity"]),
                    scales=p(ins["scales"]), rotations=p(ins["rotations"]), sh=p(ins["sh"]))
    o = A.ForwardOutputs(**{k: p(v) for k, v in outs.items()})
    nr = ctypes.c_int(-1)
    rc = lib.r3dg_rasterize_gaussians_ex(ctypes.byref(s), ctypes.byref(g), ctypes.byref(o), alloc, 1, alloc, 2, alloc,
                                         3, alloc, 4, ctypes.byref(nr), _stream())
    assert rc == 0, lib.r3dg_last_error()
    torch.cuda.synchronize()
    off = lib.r3dg_image_state_n_contrib_offset(H, W)
    outs["n_contrib"] = bufs[3][off:off + 4 * H * W].view(torch.int32).view(H, W, 1)
    return dict(outs=outs, ins=ins, s=s, g=g, geom=bufs[1], binning=bufs[2], image=bufs[3], L=nr.value)


def _raw_backward(lib, A, fwd, dc, do, dd, df, keep):
    """r3dg_rasterize_gaussians_backward through ctypes, the reference's CHW / planar gradients
    (rasterize_points.cu:183-275)."""
    import torch

    from tests._helpers import tt

    P, S, M = fwd["s"].P, fwd["s"].S, fwd["s"].M
    grads = dict(dc=tt(dc), do=tt(do), dd=tt(dd), df=tt(df))
    keep.append(grads)
    f = lambda *s: torch.empty(*s, device="cuda")  # noqa: E731
    res = dict(dL_dmeans2D=f(P, 3), dL_dcolors=f(P, 3), dL_dopacity=f(P, 1), dL_dmeans3D=f(P, 3),
               dL_dfeatures=f(P, S), dL_dcov3D=f(P, 6), dL_dsh=f(P, M, 3), dL_dscales=f(P, 3), dL_drotations=f(P, 4))
    scratch = []

    @A.ALLOC
    def alloc(ctx, n):
        t = torch.empty(max(int(n), 256), dtype=torch.uint8, device="cuda")
        scratch.append(t)
        return t.data_ptr()

    keep.append(alloc)
    p = lambda t: t.data_ptr()  # noqa: E731
    gr = A.BackwardGrads(dL_dout_color=p(grads["dc"]), color_hwc=0, dL_dout_opacity=p(grads["do"]),
                         dL_dout_depth=p(grads["dd"]), dL_dout_feature=p(grads["df"]), feature_native=0)
    out = A.new(A.BackwardOutputs, **{k: p(v) for k, v in res.items()})
    rc = lib.r3dg_rasterize_gaussians_backward(ctypes.byref(fwd["s"]), ctypes.byref(fwd["g"]),
                                               p(fwd["outs"]["radii"]), ctypes.byref(gr), p(fwd["geom"]),
                                               p(fwd["binning"]), p(fwd["image"]), fwd["L"], 1, alloc, None,
                                               ctypes.byref(out), _stream())
    assert rc == 0, lib.r3dg_last_error()
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in res.items()}


def test_hot_path_raw_ctypes(abi):
    """The hot path's C ABI as a non-torch host binds it: r3dg_rasterize_gaussians_ex
    and r3dg_rasterize_gaussians_backward through ctypes with torch-backed allocation callbacks and the
    options switched through r3dg_set_options. Forward bit-identical to the `_C` binding; backward
    bit-identical to `_C` on the deterministic rows reduction and within the oracle's GRAD_BARS on the
    default atomic flush."""
    from tests import _abi_ctypes as A
    from tests._helpers import hip_backward, hip_forward, upstream_grads
    from tests.test_gpu_parity import _check_forward, _oracle_fwd, grad_check

    import relightable3dgaussian_amd as r3

    lib = A.bind(abi)
    S = 11
    scene, cam = synthetic.small_scene(P=3000, S=21, seed=23, width=112, height=80)
    keep = []
    raw = _raw_forward(lib, A, scene, cam, S, keep)
    ref = hip_forward(r3._C, scene, cam, S=S)
    assert raw["L"] == ref["num_rendered"] > 0
    for k in ("color", "opacity", "depth", "stencil", "feature", "shader_color", "normal", "surface_xyz", "radii",
              "n_contrib"):
        np.testing.assert_array_equal(raw["outs"][k].cpu().numpy(), ref[k].cpu().numpy(), err_msg=k)
    o = _oracle_fwd(scene, cam, S)
    _check_forward(dict(raw["outs"], num_rendered=raw["L"], _cam=cam, geom=raw["geom"], binning=raw["binning"],
                        image=raw["image"]), o, S)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, S, seed=6)

    saved = A.new(A.Options)
    assert lib.r3dg_get_options(ctypes.byref(saved)) == 0
    try:
        rows = A.new(A.Options)
        ctypes.memmove(ctypes.byref(rows), ctypes.byref(saved), ctypes.sizeof(A.Options))
        rows.bwd_reduce = 1
        assert lib.r3dg_set_options(ctypes.byref(rows)) == 0
        assert r3._C.get_options()["bwd_reduce"] == 1  # one library instance behind ctypes and `_C`
        g_raw = _raw_backward(lib, A, raw, dc, do, dd, df, keep)
        g_ref = hip_backward(r3._C, ref, dc, do, dd, df)
        for k in g_ref:
            np.testing.assert_array_equal(g_raw[k], g_ref[k], err_msg=k)
        rows.bwd_reduce = 0
        assert lib.r3dg_set_options(ctypes.byref(rows)) == 0
        g_atomic = _raw_backward(lib, A, raw, dc, do, dd, df, keep)
    finally:
        assert lib.r3dg_set_options(ctypes.byref(saved)) == 0
    import oracle as orc

    grad_check("raw ctypes atomic", g_atomic, orc.rasterize_backward(o, dc, do, dd, df))
