"""CPU oracle -- TEST INFRASTRUCTURE ONLY (never imported by the product package).

numpy/ctypes front end of r3dg_oracle.c, the C restatement of the reference hot path
(see that file's header for per-function reference citations). Used by tests/, by
__graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg.

Pinning: tests/test_oracle_golden.py checks this oracle against vectors produced by the
reference's own PyTorch code (tests/golden/make_golden.py). The tile blend has no reference
fixture; DESIGN.md "Parity" explains what pins it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(HERE, "_build", "libr3dg_oracle.so")
_lib = None

F = np.float32


def build() -> str:
    srcs = [os.path.join(HERE, f) for f in ("r3dg_oracle.c", "r3dg_shaders.c", "r3dg_bvh.c", "Makefile")]
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB)
        _lib.oracle_higher_msb.restype = ctypes.c_uint32
        _lib.oracle_higher_msb.argtypes = [ctypes.c_uint32]
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be contiguous"
    return a.ctypes.data_as(ctypes.c_void_p)


def _f(a):
    return None if a is None else np.ascontiguousarray(a, dtype=F)


def feature_layout(S: int, HW: int):
    a = np.zeros(max(S, 1), np.int64)
    m = np.zeros(max(S, 1), np.int32)
    lib().oracle_feature_layout(ctypes.c_int(S), ctypes.c_longlong(HW), _p(a), _p(m))
    return a[:S], m[:S]


def planar_layout(S: int, HW: int):
    return (np.arange(S, dtype=np.int64) * HW), np.ones(S, np.int32)


# ---------------------------------------------------------------------------------------------
# textures and shaders (r3dg_shaders.c)
# ---------------------------------------------------------------------------------------------
# registry ids: the alphabetical name order of the shader maps (ShShader.cu:196-230,
# splatShader.cu:283-333), the same ids the HIP registry hands out
SH_CULLHALF, SH_EXPPOS, SH_GAUSSDISSOLVE, SH_HEARTBEAT, SH_DEFAULT = range(5)
SH_NAMES = ["CullHalf", "ExpPos", "GaussDissolve", "Heartbeat", "ShDefault"]
(SP_CRACK, SP_CRACKNORECON, SP_DISSOLVE, SP_NAIVEOUTLINE, SP_QUANTIZEFLATS, SP_QUANTIZELIGHT, SP_ROUGHNESSONLY,
 SP_DEFAULT, SP_STENCIL, SP_WIREFRAME) = range(10)
SPLAT_NAMES = ["Crack", "CrackNoRecon", "Dissolve", "NaiveOutline", "QuantizeFlats", "QuantizeLight",
               "RoughnessOnly", "SplatDefault", "Stencil", "Wireframe"]
(PP_BLURLIGHTING, PP_CRACKRECON, PP_INVERT, PP_OUTLINE, PP_QUANTIZELIGHTING, PP_SOBEL, PP_DEFAULT,
 PP_TEXTUREDSHADOWS, PP_TOON) = range(9)
POST_NAMES = ["BlurLighting", "CrackReconstriction", "Invert", "Outline", "QuantizeLighting", "SobelFilter",
              "SplatDefault", "TexturedShadows", "ToonShader"]
# textures each shader samples (TextureManager names used in ShShader.cu / splatShader.cu)
SH_TEXTURES = {SH_HEARTBEAT: ("Turbulence", "Craters"), SH_GAUSSDISSOLVE: ("Cracks", None)}
SPLAT_TEXTURES = {SP_DISSOLVE: "Cracks", SP_CRACK: "Depth cracks", SP_CRACKNORECON: "Bulge"}
# channels per TextureMode (texture.h), in r3dg_encode_texture_mode order
MODE_CHANNELS = {0: 1, 1: 1, 2: 1, 9: 1, 10: 1, 3: 3, 6: 3, 7: 3, 8: 3, 4: 4, 5: 4}
ADDR_WRAP, ADDR_CLAMP, ADDR_MIRROR, ADDR_BORDER = range(4)


class OTex(ctypes.Structure):
    _fields_ = [("texels", ctypes.c_void_p), ("W", ctypes.c_int), ("H", ctypes.c_int), ("wrap_u", ctypes.c_int),
                ("wrap_v", ctypes.c_int), ("normalized", ctypes.c_int), ("linear", ctypes.c_int)]


class Texture:
    """AllocateTexture (texture.cu:86-233) for the oracle: pixels [H, W, C] padded to float4
    texels (1 channel -> (x, 0, 0, 1), 3 channels -> alpha 1), bilinear sampling except LAB / HSV
    (modes 7, 8: point sampling)."""

    def __init__(self, pixels, mode=3, wrap_u=ADDR_WRAP, wrap_v=ADDR_WRAP, normalized=True):
        C = MODE_CHANNELS[mode]
        pix = np.asarray(pixels, F)
        H, W = pix.shape[:2]
        pix = pix.reshape(H, W, C)
        t = np.zeros((H, W, 4), F)
        t[..., 3] = 1.0
        t[..., :C] = pix
        self.texels = np.ascontiguousarray(t)
        self.pixels = pix
        self.mode, self.wrap = mode, (wrap_u, wrap_v)
        self.normalized = bool(normalized)
        self.desc = OTex(self.texels.ctypes.data, W, H, wrap_u, wrap_v, int(bool(normalized)),
                         0 if mode in (7, 8) else 1)

    def sample(self, xy):
        """tex2D<float4> at each (x, y) row of xy [n, 2] -> [n, 4]."""
        xy = _f(xy).reshape(-1, 2)
        out = np.zeros((xy.shape[0], 4), F)
        lib().oracle_tex_sample_batch(ctypes.byref(self.desc), ctypes.c_int(xy.shape[0]), _p(xy), _p(out))
        return out


def sh_shader(sid, idx, pos, scale, rot, opacity, sh, features=None, time=0.0, tex0=None, tex1=None):
    """One SH shader over the splats idx, in place on the (float32, contiguous) arrays."""
    idx = np.ascontiguousarray(idx, np.int32)
    S = 0 if features is None else features.shape[1]
    lib().oracle_sh_shader(ctypes.c_int(sid), ctypes.c_int(idx.size), _p(idx), ctypes.c_float(time), _p(pos),
                           _p(scale), _p(rot), _p(opacity), _p(sh), ctypes.c_int(sh.shape[1]), _p(features),
                           ctypes.c_int(S), ctypes.byref(tex0.desc) if tex0 else None,
                           ctypes.byref(tex1.desc) if tex1 else None)


def splat_shader(sid, idx, W, H, pos, means2D, depth_tex, view_inv, depths, rgb, conic_opacity, features, stencils,
                 stencil_opacity, out_rgb, time=0.0, tex0=None):
    """One splat shader over the splats idx, in place on conic_opacity / features / stencils /
    stencil_opacity / out_rgb."""
    idx = np.ascontiguousarray(idx, np.int32)
    lib().oracle_splat_shader(ctypes.c_int(sid), ctypes.c_int(idx.size), _p(idx), ctypes.c_int(W), ctypes.c_int(H),
                              ctypes.c_float(time), _p(pos), _p(means2D), _p(depth_tex), _p(_f(view_inv)), _p(depths),
                              _p(rgb), _p(conic_opacity), _p(features), ctypes.c_int(features.shape[1]),
                              _p(stencils), _p(stencil_opacity), _p(out_rgb),
                              ctypes.byref(tex0.desc) if tex0 else None)


# ---------------------------------------------------------------------------------------------
# rasterizer
# ---------------------------------------------------------------------------------------------
def rasterize_forward(cam, means3D, opacity, features, sh=None, degree=3, scales=None, rotations=None,
                      cov3D_precomp=None, colors_precomp=None, bg=(1.0, 1.0, 1.0), scale_modifier=1.0,
                      compute_pseudo_normal=True, sh_shaders=None, splat_shaders=None, textures=None,
                      error_texture=None, time=0.0, post_passes=None):
    """Full forward of rasterize_gaussians (rasterizer_impl.cu:213-529). Returns a dict with the
    reference outputs (HWC) and the binning state.

    Shaders (forward.cu:805-971): `sh_shaders` / `splat_shaders` are per-splat registry ids
    (SH_* / SP_* below; None = the default shaders), `textures` maps names to `Texture`s and
    `error_texture` stands in for missing names (TextureManager::GetTexture, texture.cu:298-314).
    SH shaders edit working copies of the inputs before preprocessing; splat shaders run after
    the intermediate depth / stencil pass and edit opacity, features and the shader colour.
    `post_passes` (PP_* ids, in order) re-render depth + stencil and run the screen passes
    (rasterizer_impl.cu:485-529)."""
    L_ = lib()
    means3D = _f(means3D)
    P = means3D.shape[0]
    features = _f(features) if features is not None else np.zeros((P, 0), F)
    S = features.shape[1]
    W, H = cam.width, cam.height
    gx, gy = (W + 15) // 16, (H + 15) // 16
    sh = _f(sh)
    M = 0 if sh is None else sh.shape[1]
    scales, rotations, cov3D_precomp, colors_precomp = map(_f, (scales, rotations, cov3D_precomp, colors_precomp))
    opacity = _f(opacity).reshape(P)
    sh_ids = None if sh_shaders is None else np.asarray(sh_shaders).reshape(-1)
    sp_ids = None if splat_shaders is None else np.asarray(splat_shaders).reshape(-1)
    sh_active = P > 0 and sh_ids is not None and bool((sh_ids != SH_DEFAULT).any())
    splat_active = P > 0 and sp_ids is not None and bool((sp_ids != SP_DEFAULT).any())
    originals = dict(means3D=means3D, scales=scales, rotations=rotations, sh=sh, features=features)
    if sh_active or splat_active:  # working copies (rasterize_points.cu:117-122)
        cp = lambda a: None if a is None else a.copy()  # noqa: E731
        means3D, scales, rotations, opacity, sh, features = map(cp, (means3D, scales, rotations, opacity, sh,
                                                                     features))

    def tex(name):
        if name is None:
            return None
        t = (textures or {}).get(name, error_texture)
        if t is None:
            raise ValueError(f"shader samples texture {name!r}: pass textures / error_texture")
        return ctypes.byref(t.desc)

    if sh_active:  # RunSHShaders (forward.cu:805-877)
        for sid in np.unique(sh_ids):
            if sid == SH_DEFAULT:
                continue
            idx = np.ascontiguousarray(np.nonzero(sh_ids == sid)[0], np.int32)
            t0, t1 = SH_TEXTURES.get(int(sid), (None, None))
            L_.oracle_sh_shader(ctypes.c_int(int(sid)), ctypes.c_int(idx.size), _p(idx), ctypes.c_float(time),
                                _p(means3D), _p(scales), _p(rotations), _p(opacity), _p(sh), ctypes.c_int(M),
                                _p(features), ctypes.c_int(S), tex(t0), tex(t1))
    view, proj, campos = _f(cam.view), _f(cam.proj), _f(cam.campos)
    radii = np.zeros(P, np.int32)
    means2D = np.zeros((P, 2), F)
    depths = np.zeros(P, F)
    cov3D = np.zeros((P, 6), F)
    rgb = np.zeros((P, 3), F)
    clamped = np.zeros(P, np.uint8)
    conic = np.zeros((P, 4), F)
    touched = np.zeros(P, np.uint32)
    L_.oracle_preprocess(ctypes.c_int(P), ctypes.c_int(degree), ctypes.c_int(M), _p(means3D), _p(scales),
                         ctypes.c_float(scale_modifier), _p(rotations), _p(opacity), _p(sh), _p(cov3D_precomp),
                         _p(colors_precomp), _p(view), _p(proj), _p(campos), ctypes.c_int(W), ctypes.c_int(H),
                         ctypes.c_float(cam.tanfovx), ctypes.c_float(cam.tanfovy), _p(radii), _p(means2D),
                         _p(depths), _p(cov3D), _p(rgb), _p(clamped), _p(conic), _p(touched))
    offsets = np.cumsum(touched, dtype=np.uint64).astype(np.uint32)
    L = int(offsets[-1]) if P else 0
    keys = np.zeros(max(L, 1), np.uint64)
    vals = np.zeros(max(L, 1), np.uint32)
    L_.oracle_duplicate_with_keys(ctypes.c_int(P), _p(means2D), _p(depths), _p(offsets), _p(radii), ctypes.c_int(W),
                                  ctypes.c_int(H), _p(keys), _p(vals))
    bit = L_.oracle_higher_msb(gx * gy)
    keys_s = np.zeros_like(keys)
    vals_s = np.zeros_like(vals)
    L_.oracle_sort_pairs(ctypes.c_longlong(L), _p(keys), _p(vals), _p(keys_s), _p(vals_s), ctypes.c_int(32 + bit))
    ranges = np.zeros((gx * gy, 2), np.uint32)
    L_.oracle_identify_tile_ranges(ctypes.c_longlong(L), _p(keys_s), ctypes.c_int(gx * gy), _p(ranges))
    colors = colors_precomp if colors_precomp is not None else rgb
    bgv = np.asarray(bg, F)
    HW = H * W
    stencil_img = np.zeros((H, W, 1), F)
    shader_rgb = colors
    stencils = np.zeros(P, F)          # InitializeStencil (rasterizer_impl.cu:203-209)
    stencil_opacity = np.ones(P, F)
    if splat_active:
        # RenderIntermediateTextures (forward.cu:271-383), then RunSplatShaders (forward.cu:907-971)
        depth_img = np.zeros((H, W, 1), F)
        L_.oracle_render_intermediate(ctypes.c_int(W), ctypes.c_int(H), _p(ranges), _p(vals_s), _p(means2D),
                                      _p(depths), _p(stencils), _p(conic), _p(stencil_opacity), _p(depth_img),
                                      _p(stencil_img))
        shader_rgb = np.zeros((P, 3), F)
        vinv = _f(cam.view_inv)
        for sid in np.unique(sp_ids):
            idx = np.ascontiguousarray(np.nonzero(sp_ids == sid)[0], np.int32)
            L_.oracle_splat_shader(ctypes.c_int(int(sid)), ctypes.c_int(idx.size), _p(idx), ctypes.c_int(W),
                                   ctypes.c_int(H), ctypes.c_float(time), _p(means3D), _p(means2D), _p(depth_img),
                                   _p(vinv), _p(depths), _p(colors), _p(conic), _p(features), ctypes.c_int(S),
                                   _p(stencils), _p(stencil_opacity), _p(shader_rgb),
                                   tex(SPLAT_TEXTURES.get(int(sid))))
    final_T = np.zeros(HW, F)
    n_contrib = np.zeros(HW, np.uint32)
    out_color = np.zeros((H, W, 3), F)
    out_shader = np.zeros((H, W, 3), F)
    out_opacity = np.zeros((H, W, 1), F)
    out_depth = np.zeros((H, W, 1), F)
    out_feature = np.zeros((H, W, S), F)
    L_.oracle_render_forward(ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(S), _p(ranges), _p(vals_s),
                             _p(means2D), _p(depths), _p(features), _p(shader_rgb), _p(colors), _p(conic), _p(bgv),
                             _p(final_T), _p(n_contrib), _p(out_color), _p(out_opacity), _p(out_depth),
                             _p(out_feature), _p(out_shader))
    normal = np.zeros((H, W, 3), F)
    xyz = np.zeros((H, W, 3), F)
    if compute_pseudo_normal:
        fx, fy = cam.focal
        L_.oracle_surface_xyz_normal(ctypes.c_int(W), ctypes.c_int(H), _p(view), ctypes.c_float(fx),
                                     ctypes.c_float(fy), ctypes.c_float(cam.cx), ctypes.c_float(cam.cy),
                                     _p(out_opacity), _p(out_depth), _p(normal), _p(xyz))
    if post_passes is not None and len(post_passes) > 0:
        # rasterizer_impl.cu:485-529: depth + stencil rendered again, then RunPostProcessShaders
        L_.oracle_render_intermediate(ctypes.c_int(W), ctypes.c_int(H), _p(ranges), _p(vals_s), _p(means2D),
                                      _p(depths), _p(stencils), _p(conic), _p(stencil_opacity), _p(out_depth),
                                      _p(stencil_img))
        ids = np.ascontiguousarray(post_passes, np.int32)
        needs_shadow = bool(np.isin(ids, [PP_TEXTUREDSHADOWS, PP_TOON]).any())
        L_.oracle_post_passes(_p(ids), ctypes.c_int(ids.size), ctypes.c_int(W), ctypes.c_int(H), _p(view),
                              _p(out_color), _p(out_opacity), _p(out_depth), _p(stencil_img), _p(xyz), _p(normal),
                              _p(out_feature) if S == 21 else None, _p(out_shader),
                              tex("shadow") if needs_shadow else None)
    return dict(num_rendered=L, color=out_color, opacity=out_opacity, depth=out_depth,
                stencil=stencil_img, feature=out_feature, shader_color=out_shader, normal=normal,
                surface_xyz=xyz, radii=radii, n_contrib=n_contrib.reshape(H, W, 1), final_T=final_T,
                keys=keys_s[:L], point_list=vals_s[:L], ranges=ranges, offsets=offsets, depths=depths,
                means2D=means2D, conic_opacity=conic, rgb=rgb, clamped=clamped, cov3D=cov3D,
                # inputs kept for the backward
                # the backward reads the caller's tensors, not the shaded copies (rasterize_points.cu)
                _in=dict(means3D=originals["means3D"], features=originals["features"], sh=originals["sh"],
                         degree=degree, scales=originals["scales"], rotations=originals["rotations"],
                         cov3D_precomp=cov3D_precomp, colors_precomp=colors_precomp, scale_modifier=scale_modifier, bg=bgv, cam=cam))


def rasterize_backward(fwd, dL_dcolor, dL_dopacity, dL_ddepth, dL_dfeature, color_hwc=False, feature_native=False,
                       backward_geometry=True, acc64=False):
    """rasterize_gaussians_backward (rasterizer_impl.cu:533-639). Grad layouts: colour CHW [3,H,W]
    (reference) unless color_hwc; features planar [S,H,W] (reference) unless feature_native.
    acc64 (test-only accuracy reference, not the reference's arithmetic): the per-pixel mean2D /
    conic / opacity terms formed in double and summed in double, rounded to f32 once, then the same
    f32 per-Gaussian backward."""
    L_ = lib()
    i = fwd["_in"]
    cam = i["cam"]
    W, H = cam.width, cam.height
    HW = H * W
    P = i["means3D"].shape[0]
    S = i["features"].shape[1]
    if color_hwc:
        ca, cm = np.arange(3, dtype=np.int64), np.full(3, 3, np.int32)
    else:
        ca, cm = np.arange(3, dtype=np.int64) * HW, np.ones(3, np.int32)
    fa, fm = feature_layout(S, HW) if feature_native else planar_layout(S, HW)
    fa = np.ascontiguousarray(fa if S else np.zeros(1, np.int64))
    fm = np.ascontiguousarray(fm if S else np.zeros(1, np.int32))
    colors = i["colors_precomp"] if i["colors_precomp"] is not None else fwd["rgb"]
    dmean2D = np.zeros((P, 3), F)
    dconic = np.zeros((P, 4), F)
    dopac = np.zeros((P, 1), F)
    dcol = np.zeros((P, 3), F)
    dfeat = np.zeros((P, S), F)
    gc, go, gd = _f(dL_dcolor), _f(dL_dopacity), _f(dL_ddepth)
    gf = _f(dL_dfeature) if S else np.zeros(1, F)
    if acc64:
        a64 = [np.zeros((P, 3)), np.zeros((P, 4)), np.zeros((P, 1))]
        L_.oracle_set_render_bwd_acc64(*[a.ctypes.data_as(ctypes.c_void_p) for a in a64])
    L_.oracle_render_backward(ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(S), _p(fwd["ranges"]),
                              _p(np.ascontiguousarray(fwd["point_list"])), _p(i["bg"]), _p(fwd["means2D"]),
                              _p(fwd["depths"]), _p(fwd["conic_opacity"]), _p(colors), _p(i["features"]),
                              _p(fwd["final_T"]), _p(np.ascontiguousarray(fwd["n_contrib"].reshape(-1))), _p(gc),
                              _p(ca), _p(cm), _p(go), _p(gd), _p(gf), _p(fa), _p(fm), ctypes.c_int(int(backward_geometry)),
                              _p(dmean2D), _p(dconic), _p(dopac), _p(dcol), _p(dfeat))
    if acc64:
        L_.oracle_set_render_bwd_acc64(None, None, None)
        dmean2D[:] = a64[0].astype(F)
        dconic[:] = a64[1].astype(F)
        dopac[:] = a64[2].astype(F)
    M = 0 if i["sh"] is None else i["sh"].shape[1]
    dmean3D = np.zeros((P, 3), F)
    dcov = np.zeros((P, 6), F)
    dsh = np.zeros((P, M, 3), F)
    dscale = np.zeros((P, 3), F)
    drot = np.zeros((P, 4), F)
    cov = i["cov3D_precomp"] if i["cov3D_precomp"] is not None else fwd["cov3D"]
    L_.oracle_preprocess_backward(ctypes.c_int(P), ctypes.c_int(i["degree"]), ctypes.c_int(M), _p(i["means3D"]),
                                  _p(fwd["radii"]), _p(i["sh"]), _p(fwd["clamped"]), _p(i["scales"]),
                                  _p(i["rotations"]), ctypes.c_float(i["scale_modifier"]), _p(cov),
                                  _p(_f(cam.view)), _p(_f(cam.proj)), ctypes.c_int(W), ctypes.c_int(H),
                                  ctypes.c_float(cam.tanfovx), ctypes.c_float(cam.tanfovy), _p(_f(cam.campos)),
                                  _p(dmean2D), _p(dconic), _p(dcol), _p(dmean3D), _p(dcov), _p(dsh), _p(dscale),
                                  _p(drot))
    return dict(dL_dmeans2D=dmean2D, dL_dcolors=dcol, dL_dopacity=dopac, dL_dmeans3D=dmean3D, dL_dfeatures=dfeat,
                dL_dcov3D=dcov, dL_dsh=dsh, dL_dscales=dscale, dL_drotations=drot, dL_dconic=dconic)


def expf(x):
    """r3dg_expf, the blend's exp (forward.cu:477 / backward.cu:527), elementwise on float32."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    f = lib().r3dg_expf
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_float]
    return np.array([f(float(v)) for v in x], np.float32)


def expf_wide(x):
    """r3dg_expf_wide, the render equation's exp (render_equation.cu:151 / :351), elementwise."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    f = lib().r3dg_expf_wide
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_float]
    return np.array([f(float(v)) for v in x], np.float32)


def sincosf(x):
    """r3dg_sincosf, the Fibonacci angle's sin / cos (render_equation.cu:93-94): (sin, cos)."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    f = lib().r3dg_sincosf
    f.restype = None
    f.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    s, c = ctypes.c_float(), ctypes.c_float()
    out = np.empty((2, x.size), np.float32)
    for i, v in enumerate(x):
        f(float(v), ctypes.byref(s), ctypes.byref(c))
        out[0, i], out[1, i] = s.value, c.value
    return out[0], out[1]


class blend_exp_libm:
    """Context manager: the oracle's blend uses glibc expf instead of r3dg_expf (measures the exp
    choice; the HIP kernels always use r3dg_expf)."""

    def __enter__(self):
        lib().oracle_set_blend_exp(ctypes.c_int(1))
        return self

    def __exit__(self, *exc):
        lib().oracle_set_blend_exp(ctypes.c_int(0))
        return False


class power_ref_ops:
    """Context manager: the oracle's blend evaluates the Gaussian's power with the reference's
    operation order (forward.cu:478; mode 1 as written, mode 2 with nvcc's default contractions)
    instead of the staged FMA pattern the HIP kernels share with it (measures that choice,
    DESIGN.md §5)."""

    def __init__(self, mode=1):
        self.mode = mode

    def __enter__(self):
        lib().oracle_set_power_ref_ops(ctypes.c_int(self.mode))
        return self

    def __exit__(self, *exc):
        lib().oracle_set_power_ref_ops(ctypes.c_int(0))
        return False


def expf_accuracy(lo=-80.0, hi=0.0, stride=1):
    """(max ulp error, n, correctly rounded count) of r3dg_expf against double exp over every
    `stride`-th float in [lo, hi]."""
    f = lib().oracle_expf_max_ulp
    f.restype = ctypes.c_double
    n, ex = ctypes.c_longlong(0), ctypes.c_longlong(0)
    m = f(ctypes.c_float(lo), ctypes.c_float(hi), ctypes.c_uint32(stride), ctypes.byref(n), ctypes.byref(ex))
    return m, n.value, ex.value


def mark_visible(means3D, view):
    means3D = _f(means3D)
    out = np.zeros(means3D.shape[0], np.uint8)
    lib().oracle_mark_visible(ctypes.c_int(means3D.shape[0]), _p(means3D), _p(_f(view)), _p(out))
    return out.astype(bool)


def color_from_sh(means, campos, shs, degree):
    """computeColorFromSH (forward.cu:25-76): (rgb [P,3], clamped bits [P])."""
    means, campos, shs = _f(means), _f(campos), _f(shs)
    P, M = shs.shape[0], shs.shape[1]
    rgb = np.zeros((P, 3), F)
    cl = np.zeros(P, np.uint8)
    lib().oracle_color_from_sh_batch(ctypes.c_int(P), ctypes.c_int(degree), ctypes.c_int(M), _p(means), _p(campos),
                                     _p(shs), _p(rgb), _p(cl))
    return rgb, cl


def cov3d(scales, rotations, scale_modifier=1.0):
    """computeCov3D (forward.cu:124-158): upper triangle [P,6]."""
    scales, rotations = _f(scales), _f(rotations)
    out = np.zeros((scales.shape[0], 6), F)
    lib().oracle_cov3d_batch(ctypes.c_int(scales.shape[0]), _p(scales), ctypes.c_float(scale_modifier),
                             _p(rotations), _p(out))
    return out


# ---------------------------------------------------------------------------------------------
# BRDF
# ---------------------------------------------------------------------------------------------
def _brdf_args(inp):
    b = {k: _f(v) for k, v in inp.items()}
    P = b["base"].shape[0]
    Si, Sd, Sv = b["incidents"].shape[1], b["env"].shape[1], b["visibility"].shape[1]
    if max(Si, Sd, Sv) > 16:  # computeSHcoef (render_equation.cu:17-50) yields 16 coefficients
        raise ValueError(f"render equation: SH coefficient counts must be <= 16 (got {Si}, {Sd}, {Sv})")
    return b, P, Si, Sd, Sv


class brdf_reference_ops:
    """Context manager: the oracle's render equation evaluates the reference's own operation
    sequence (render_equation.cu: libm sinf / cosf / expf / powf, every division as written) instead
    of the shared statements brdf.hip restates bit for bit (oracle/r3dg_oracle.c g_brdf_ref_ops)."""

    def __enter__(self):
        lib().oracle_set_brdf_ref_ops(ctypes.c_int(1))
        return self

    def __exit__(self, *exc):
        lib().oracle_set_brdf_ref_ops(ctypes.c_int(0))
        return False


def brdf_forward(inp, sample_num=24, is_training=False, rand=None):
    b, P, Si, Sd, Sv = _brdf_args(inp)
    dirs = np.zeros((P, sample_num, 3), F)
    pbr = np.zeros((P, 3), F)
    diff = np.zeros((P, 3), F)
    rnd = _f(rand).reshape(P, sample_num) if rand is not None else None
    lib().oracle_render_equation_forward(ctypes.c_int(P), ctypes.c_int(Si), ctypes.c_int(Sd), ctypes.c_int(Sv),
                                         _p(b["base"]), _p(b["rough"]), _p(b["metal"]), _p(b["normals"]),
                                         _p(b["viewdirs"]), _p(b["incidents"]), _p(b["env"]), _p(b["visibility"]),
                                         ctypes.c_int(sample_num), ctypes.c_int(int(is_training)), _p(rnd),
                                         _p(dirs), _p(pbr), _p(diff))
    return dict(pbr=pbr, incident_dirs=dirs, diffuse_light=diff)


def brdf_forward_complex(inp, sample_num=24):
    b, P, Si, Sd, Sv = _brdf_args(inp)
    Ns = sample_num
    o = dict(incident_dirs=np.zeros((P, Ns, 3), F), pbr=np.zeros((P, 3), F),
             incident_lights=np.zeros((P, Ns, 3), F), local_incident_lights=np.zeros((P, Ns, 3), F),
             global_incident_lights=np.zeros((P, Ns, 3), F), incident_visibility=np.zeros((P, Ns, 1), F),
             diffuse_light=np.zeros((P, 3), F), local_diffuse_light=np.zeros((P, 3), F), accum=np.zeros((P, 1), F),
             rgb_d=np.zeros((P, 3), F), rgb_s=np.zeros((P, 3), F))
    lib().oracle_render_equation_forward_complex(
        ctypes.c_int(P), ctypes.c_int(Si), ctypes.c_int(Sd), ctypes.c_int(Sv), _p(b["base"]), _p(b["rough"]),
        _p(b["metal"]), _p(b["normals"]), _p(b["viewdirs"]), _p(b["incidents"]), _p(b["env"]), _p(b["visibility"]),
        ctypes.c_int(Ns), _p(o["incident_dirs"]), _p(o["pbr"]), _p(o["incident_lights"]),
        _p(o["local_incident_lights"]), _p(o["global_incident_lights"]), _p(o["incident_visibility"]),
        _p(o["diffuse_light"]), _p(o["local_diffuse_light"]), _p(o["accum"]), _p(o["rgb_d"]), _p(o["rgb_s"]))
    return o


def brdf_backward(inp, incident_dirs, dL_dpbr, dL_ddiffuse, sample_num=24):
    b, P, Si, Sd, Sv = _brdf_args(inp)
    o = dict(base=np.zeros((P, 3), F), rough=np.zeros((P, 1), F), metal=np.zeros((P, 1), F),
             normals=np.zeros((P, 3), F), viewdirs=np.zeros((P, 3), F), incidents=np.zeros((P, Si, 3), F),
             env=np.zeros((1, Sd, 3), F), visibility=np.zeros((P, Sv, 1), F))
    lib().oracle_render_equation_backward(
        ctypes.c_int(P), ctypes.c_int(Si), ctypes.c_int(Sd), ctypes.c_int(Sv), _p(b["base"]), _p(b["rough"]),
        _p(b["metal"]), _p(b["normals"]), _p(b["viewdirs"]), _p(b["incidents"]), _p(b["env"]), _p(b["visibility"]),
        ctypes.c_int(sample_num), _p(_f(incident_dirs)), _p(_f(dL_dpbr)), _p(_f(dL_ddiffuse)), _p(o["base"]),
        _p(o["rough"]), _p(o["metal"]), _p(o["normals"]), _p(o["viewdirs"]), _p(o["incidents"]), _p(o["env"]),
        _p(o["visibility"]))
    return o


# ---- BVH visibility tracer (r3dg_bvh.c; reference bvh/src/*.cu, bvh/__init__.py) -------------

def bvh_leaf_aabbs(means3D, scales, rotations):
    m, s, r = _f(means3D), _f(scales), _f(rotations)
    P = m.shape[0]
    out = np.zeros((P, 6), F)
    lib().oracle_bvh_leaf_aabbs(ctypes.c_int(P), _p(m), _p(s), _p(r), _p(out))
    return out


def bvh_build(leaf_aabbs):
    """create_bvh on leaf boxes in Gaussian order -> (nodes int32 [2P-1,5], aabbs [2P-1,6], morton u64 [P])."""
    leaf = _f(leaf_aabbs)
    P = leaf.shape[0]
    nodes = np.full((2 * P - 1, 5), -1, np.int32)
    aabbs = np.zeros((2 * P - 1, 6), F)
    aabbs[P - 1:] = leaf
    keys = np.zeros(P, np.uint64)
    rc = lib().oracle_bvh_build(ctypes.c_int(P), _p(nodes), _p(aabbs), _p(keys))
    assert rc == 0, "oracle_bvh_build failed"
    return nodes, aabbs, keys


def bvh_trace_opacity(nodes, aabbs, rays_o, rays_d, means3D, cov_inv, opacity, normals, with_terms=False):
    """trace_bvh_opacity -> (contribute int32 [R], visibility f32 [R], transmittance before the cut [R]
    [, factors multiplied into it int32 [R] when with_terms])."""
    o, d = _f(rays_o).reshape(-1, 3), _f(rays_d).reshape(-1, 3)
    R = o.shape[0]
    contrib = np.zeros(R, np.int32)
    vis = np.ones(R, F)
    t_last = np.ones(R, F)
    nterms = np.zeros(R, np.int32)
    lib().oracle_bvh_trace_opacity(ctypes.c_int(R), _p(np.ascontiguousarray(nodes, np.int32)), _p(_f(aabbs)), _p(o),
                                   _p(d), _p(_f(means3D)), _p(_f(cov_inv)), _p(_f(opacity).reshape(-1)),
                                   _p(_f(normals)), _p(contrib), _p(vis), _p(t_last), _p(nterms))
    return (contrib, vis, t_last, nterms) if with_terms else (contrib, vis, t_last)


def bvh_trace(nodes, aabbs, rays_o, rays_d, means3D):
    """trace_bvh -> (contribute int32 [R], point [L], position [L,3], ray_id [L])."""
    nd, bx, o, d, m = (np.ascontiguousarray(nodes, np.int32), _f(aabbs), _f(rays_o).reshape(-1, 3),
                       _f(rays_d).reshape(-1, 3), _f(means3D))
    R = o.shape[0]
    contrib = np.zeros(R, np.int32)
    lib().oracle_bvh_trace.restype = ctypes.c_long
    L = lib().oracle_bvh_trace(ctypes.c_int(R), _p(nd), _p(bx), _p(o), _p(d), _p(m), _p(contrib), None, None, None)
    point = np.zeros(max(L, 1), np.int32)
    pos = np.zeros((max(L, 1), 3), F)
    rid = np.zeros(max(L, 1), np.int32)
    L2 = lib().oracle_bvh_trace(ctypes.c_int(R), _p(nd), _p(bx), _p(o), _p(d), _p(m), _p(contrib), _p(point),
                                _p(pos), _p(rid))
    assert L2 == L
    return contrib, point[:L], pos[:L], rid[:L]
