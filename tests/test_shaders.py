"""Shader library and textures: the C oracle's sampler and shaders on the
CPU, and the HIP shader path (through _C: AllocateTexture / UploadTexturesToDevice /
create_shader_manager / rasterize_gaussians) against that oracle on the GPU.

Textures are the reference's own images (tests/golden/textures.npz, written by
tests/golden/make_textures.py from textures/*.png). The sampler follows the CUDA texture-unit
rules the reference relies on (texture.cu:148-215: normalized coordinates, wrap / clamp / mirror /
border, bilinear weights in 8-bit fixed point, point sampling for LAB / HSV); the weight
quantisation is the documented hardware behaviour, not something the reference's files pin
(parity unpinned for the sub-1/256 interpolation detail; DESIGN.md "Shaders").

Image tolerances are the north_star's 1e-4 abs fp32; per-splat shader outputs are compared at
1e-5 (transcendentals: device sinf/cosf/powf against glibc).
"""
from __future__ import annotations

import math
import os

import numpy as np
import pytest

import oracle
from relightable3dgaussian_amd import synthetic
from tests._helpers import assert_close, hip_backward, hip_forward, upstream_grads

HERE = os.path.dirname(os.path.abspath(__file__))
IMG_ATOL = 1e-4


def golden_textures():
    z = np.load(os.path.join(HERE, "golden", "textures.npz"))
    # TF.to_tensor: uint8 / 255 as float32, [H, W, C] after the permute (textureImport.py:19)
    return {k: (z[k].astype(np.float32) / np.float32(255.0)) for k in z.files}


# ---------------------------------------------------------------------------------------------
# sampler (CPU)
# ---------------------------------------------------------------------------------------------
def _np_index(i, n, mode, normalized):
    zero = np.zeros(i.shape, bool)
    if mode == oracle.ADDR_BORDER:
        zero = (i < 0) | (i >= n)
        return np.clip(i, 0, n - 1), zero
    if normalized and mode == oracle.ADDR_WRAP:
        return np.mod(i, n), zero
    if normalized and mode == oracle.ADDR_MIRROR:
        r = np.mod(i, 2 * n)
        return np.where(r < n, r, 2 * n - 1 - r), zero
    return np.clip(i, 0, n - 1), zero


def _np_sample(tex: oracle.Texture, xy):
    """Independent numpy statement of the texture-unit sampling rules."""
    t = tex.texels
    H, W = t.shape[:2]
    xy = np.asarray(xy, np.float32)
    u, v = xy[:, 0], xy[:, 1]
    if tex.normalized:
        u, v = u * np.float32(W), v * np.float32(H)

    def fetch(i, j):
        x, zx = _np_index(i, W, tex.wrap[0], tex.normalized)
        y, zy = _np_index(j, H, tex.wrap[1], tex.normalized)
        return np.where((zx | zy)[:, None], np.float32(0), t[y, x])

    if tex.mode in (7, 8):
        return fetch(np.floor(u).astype(np.int64), np.floor(v).astype(np.int64))
    ub, vb = u - np.float32(0.5), v - np.float32(0.5)
    fu, fv = np.floor(ub), np.floor(vb)
    a = (np.rint((ub - fu) * np.float32(256)) * np.float32(1 / 256))[:, None]
    b = (np.rint((vb - fv) * np.float32(256)) * np.float32(1 / 256))[:, None]
    i, j = fu.astype(np.int64), fv.astype(np.int64)
    one = np.float32(1)
    return ((one - a) * (one - b) * fetch(i, j) + a * (one - b) * fetch(i + 1, j) + (one - a) * b * fetch(i, j + 1)
            + a * b * fetch(i + 1, j + 1))


def test_texture_known_answers():
    # 2x1 single-channel ramp, texel coordinates, clamp: the bilinear weight is quantised to 1/256
    t = oracle.Texture(np.array([[0.0, 1.0]], np.float32).reshape(1, 2, 1), mode=10, wrap_u=oracle.ADDR_CLAMP,
                       wrap_v=oracle.ADDR_CLAMP, normalized=False)
    got = t.sample([[0.5 + 1 / 3, 0.5], [0.5, 0.5], [1.5, 0.5], [1.0, 0.5], [-3.0, 0.5], [9.0, 0.5]])
    np.testing.assert_array_equal(got[:, 0], [85 / 256, 0.0, 1.0, 0.5, 0.0, 1.0])
    np.testing.assert_array_equal(got[:, 1:3], 0.0)   # 1-channel: (x, 0, 0, 1)
    np.testing.assert_array_equal(got[:, 3], 1.0)
    # normalized wrap: u and u + 1 sample the same texel mix; border gives zeros outside
    rgb = np.arange(4 * 4 * 3, dtype=np.float32).reshape(4, 4, 3) / 48
    w = oracle.Texture(rgb, mode=3)
    xy = np.array([[0.3, 0.7], [0.9, 0.1]], np.float32)
    np.testing.assert_array_equal(w.sample(xy), w.sample(xy + 1))
    b = oracle.Texture(rgb, mode=3, wrap_u=oracle.ADDR_BORDER, wrap_v=oracle.ADDR_BORDER)
    np.testing.assert_array_equal(b.sample([[-0.5, 0.5], [0.5, 1.7]]), 0.0)
    # texel centres reproduce the texels exactly (RGB: alpha 1)
    c = (np.array([[1, 2]]) + 0.5) / 4
    np.testing.assert_array_equal(w.sample(c)[0], np.r_[rgb[2, 1], 1.0])
    # LAB / HSV: point sampling
    p = oracle.Texture(rgb, mode=8)
    np.testing.assert_array_equal(p.sample([[0.49, 0.26]])[0], np.r_[rgb[1, 1], 1.0])


@pytest.mark.parametrize("mode", [1, 3, 4, 7])
@pytest.mark.parametrize("wrap", [0, 1, 2, 3])
@pytest.mark.parametrize("normalized", [True, False])
def test_texture_sampler_matches_numpy(mode, wrap, normalized):
    rng = np.random.default_rng(mode * 31 + wrap * 7 + normalized)
    C = oracle.MODE_CHANNELS[mode]
    t = oracle.Texture(rng.uniform(0, 1, (5, 7, C)).astype(np.float32), mode=mode, wrap_u=wrap, wrap_v=(wrap + 1) % 4,
                       normalized=normalized)
    lo, hi = (-1.5, 2.5) if normalized else (-4.0, 11.0)
    xy = rng.uniform(lo, hi, (4096, 2)).astype(np.float32)
    np.testing.assert_allclose(t.sample(xy), _np_sample(t, xy), rtol=0, atol=2e-7)


# ---------------------------------------------------------------------------------------------
# shaders (CPU)
# ---------------------------------------------------------------------------------------------
def shader_scene(P=3000, seed=0, width=96, height=72):
    """small_scene moved 3 units down z so the splats straddle the shaders' world-space
    thresholds (Crack's projection height 2, CullHalf's x = 0, GaussDissolve's loading front)."""
    scene, _ = synthetic.small_scene(P=P, S=21, seed=seed, width=width, height=height)
    fovy = math.radians(50)
    fovx = 2 * math.atan(math.tan(fovy / 2) * width / height)
    R, T = synthetic.look_at((0.15, -0.1, -3.2), (0.0, 0.0, 1.0))
    cam = synthetic.make_camera(R, T, fovx, fovy, width, height)
    scene.means3D[:, 2] -= 3.0
    return scene, cam


def _copies(scene):
    return (scene.means3D.copy(), scene.scales.copy(), scene.rotations.copy(), scene.opacity.reshape(-1).copy(),
            scene.sh.copy())


def test_sh_shader_formulas():
    scene, _ = shader_scene(P=500, seed=2)
    pos, scale, rot, opac, sh = _copies(scene)
    idx = np.arange(0, 500, 2)
    oracle.sh_shader(oracle.SH_EXPPOS, idx, pos, scale, rot, opac, sh)
    m, s = scene.means3D[idx], scene.scales[idx]
    y = np.abs(m[:, 1])
    np.testing.assert_array_equal(pos[idx], np.stack([m[:, 0] * y * y, m[:, 1] * 2 * y, m[:, 2] * y], 1))
    np.testing.assert_array_equal(scale[idx], np.stack([s[:, 0] * y * y, s[:, 1] * 2 * y, s[:, 2] * y], 1))
    np.testing.assert_array_equal(pos[1::2], scene.means3D[1::2])        # untouched outside the bucket
    pos, scale, rot, opac, sh = _copies(scene)
    oracle.sh_shader(oracle.SH_CULLHALF, np.arange(500), pos, scale, rot, opac, sh)
    neg = scene.means3D[:, 0] < 0
    np.testing.assert_array_equal(opac[neg], 0.0)
    np.testing.assert_array_equal(scale[neg], 0.0)
    np.testing.assert_array_equal(opac[~neg], scene.opacity.reshape(-1)[~neg])


def test_gauss_dissolve_and_heartbeat_move_splats():
    scene, _ = shader_scene(P=400, seed=3)
    tex = golden_textures()
    T = {k: oracle.Texture(v, mode=4) for k, v in tex.items()}
    pos, scale, rot, opac, sh = _copies(scene)
    idx = np.arange(400)
    oracle.sh_shader(oracle.SH_GAUSSDISSOLVE, idx, pos, scale, rot, opac, sh, time=9000.0, tex0=T["Cracks"])
    # loading progress lp in [0,1]: opacity scales by lp^3, the DC colour blends toward (0.6, 0.9, 1)
    assert (opac <= scene.opacity.reshape(-1) + 1e-7).all()
    lp = np.cbrt(np.clip(opac / scene.opacity.reshape(-1), 0, 1))
    done = lp > 0.999
    assert done.any() and (~done).any()
    pos, scale, rot, opac, sh = _copies(scene)
    feats = np.ascontiguousarray(scene.features)
    oracle.sh_shader(oracle.SH_HEARTBEAT, idx, pos, scale, rot, opac, sh, features=feats, time=400.0,
                     tex0=T["Turbulence"], tex1=T["Craters"])
    d = pos - scene.means3D
    assert np.abs(d).max() > 0
    # the displacement is along the stored normal (features 6..8)
    n = feats[:, 6:9]
    cross = np.cross(d, n)
    assert np.abs(cross).max() < 1e-5


def test_cullhalf_render_equals_removal():
    scene, cam = shader_scene(P=2500, seed=5)
    ids = np.full(scene.P, oracle.SH_CULLHALF)
    a = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh,
                                 scales=scene.scales, rotations=scene.rotations, sh_shaders=ids)
    keep = scene.means3D[:, 0] >= 0
    b = oracle.rasterize_forward(cam, scene.means3D[keep], scene.opacity[keep], scene.features[keep],
                                 sh=scene.sh[keep], scales=scene.scales[keep], rotations=scene.rotations[keep])
    for k in ["color", "opacity", "depth", "feature"]:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_default_managers_are_the_default_path():
    scene, cam = shader_scene(P=1500, seed=6)
    kw = dict(sh=scene.sh, scales=scene.scales, rotations=scene.rotations)
    a = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, **kw)
    b = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, **kw,
                                 sh_shaders=np.full(scene.P, oracle.SH_DEFAULT),
                                 splat_shaders=np.full(scene.P, oracle.SP_DEFAULT))
    # an active splat manager whose shaders only copy the colour (Stencil) changes nothing visible
    ids = np.full(scene.P, oracle.SP_DEFAULT)
    ids[::3] = oracle.SP_STENCIL
    c = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, **kw, splat_shaders=ids)
    for k in ["color", "opacity", "depth", "feature", "shader_color", "stencil"]:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a[k], c[k], err_msg=k)


def test_splat_shader_colour_goes_to_shader_image_only():
    """Splat shaders write geomState.shader_rgb: out_color keeps the SH colour, out_shader_color
    blends the shaded one (FORWARD::render arguments, rasterizer_impl.cu:436-456)."""
    scene, cam = shader_scene(P=1500, seed=9)
    kw = dict(sh=scene.sh, scales=scene.scales, rotations=scene.rotations)
    a = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, **kw)
    b = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, **kw,
                                 splat_shaders=np.full(scene.P, oracle.SP_WIREFRAME))
    for k in ["color", "opacity", "depth", "feature"]:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert np.abs(a["shader_color"] - b["shader_color"]).max() > 0.1


def test_roughness_only_and_quantize_light():
    scene, cam = shader_scene(P=1000, seed=8)
    P = scene.P
    feats = np.ascontiguousarray(scene.features.copy())
    conic = np.zeros((P, 4), np.float32)
    conic[:, 3] = 0.5
    st, so, out = np.zeros(P, np.float32), np.ones(P, np.float32), np.full((P, 3), -1, np.float32)
    z = np.zeros(P, np.float32)
    args = (cam.width, cam.height, scene.means3D, np.zeros((P, 2), np.float32), np.zeros(cam.width * cam.height,
            np.float32), cam.view_inv, z, np.ones((P, 3), np.float32), conic, feats, st, so, out)
    oracle.splat_shader(oracle.SP_ROUGHNESSONLY, np.arange(P), *args)
    np.testing.assert_array_equal(feats[:, 0], np.where(scene.means3D[:, 0] < 0, 0.25, 0.75))
    np.testing.assert_array_equal(feats[:, 1:3], 0.0)
    np.testing.assert_array_equal(out, 0.0)
    feats[:] = scene.features
    oracle.splat_shader(oracle.SP_QUANTIZELIGHT, np.arange(P), *args)
    q = np.round(scene.features[:, 12:15] * np.float32(3)) / np.float32(3)
    np.testing.assert_array_equal(feats[:, 0], q.max(1))
    np.testing.assert_array_equal(out, scene.features[:, 9:12])


# ---------------------------------------------------------------------------------------------
# GPU parity: HIP shader path vs the oracle
# ---------------------------------------------------------------------------------------------
def _gpu_textures(hip_ext, tex):
    import torch

    handles = {}
    for name, pix in tex.items():
        H, W = pix.shape[:2]
        d = {"pixelData": torch.tensor(pix, device="cuda"),
             "height": torch.tensor([H], dtype=torch.int32), "width": torch.tensor([W], dtype=torch.int32),
             "encoding_mode": torch.tensor([hip_ext.EncodeTextureMode("RGBA")], dtype=torch.int32),
             "wrap_modes": torch.tensor([hip_ext.EncodeWrapMode("Wrap")] * 2, dtype=torch.int32),
             "normalizedCoords": torch.tensor([1], dtype=torch.int32)}
        handles[name] = hip_ext.AllocateTexture(d)
    names = list(handles)
    return hip_ext.UploadTexturesToDevice(names, [handles[n] for n in names], handles["Error"])


def _manager(hip_ext, kind, ids):
    import torch

    m = hip_ext.GetShShaderAddressMap() if kind == 0 else hip_ext.GetSplatShaderAddressMap()
    names = oracle.SH_NAMES if kind == 0 else oracle.SPLAT_NAMES
    return hip_ext.create_shader_manager(kind, torch.tensor([m[names[i]] for i in ids], dtype=torch.int64))


def _check(h, o, extra=()):
    for k in ["color", "opacity", "depth", "shader_color", "stencil", *extra]:
        assert_close(k, h[k].cpu().numpy(), o[k], IMG_ATOL)
    assert_close("feature", h["feature"].cpu().numpy().reshape(-1), o["feature"].reshape(-1), IMG_ATOL)
    np.testing.assert_array_equal(h["radii"].cpu().numpy(), o["radii"])
    assert h["num_rendered"] == o["num_rendered"]


@pytest.mark.gpu
@pytest.mark.parametrize("time", [400.0, 9000.0])
def test_sh_shaders_match_oracle(hip_ext, time):
    scene, cam = shader_scene(P=4000, seed=11)
    tex = golden_textures()
    rng = np.random.default_rng(int(time))
    ids = rng.integers(0, 5, scene.P)
    texm = _gpu_textures(hip_ext, tex)
    h = hip_forward(hip_ext, scene, cam, time=time, texture_manager=texm, sh_manager=_manager(hip_ext, 0, ids))
    T = {k: oracle.Texture(v, mode=4) for k, v in tex.items()}
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations, sh_shaders=ids, textures=T, error_texture=T["Error"],
                                 time=time)
    _check(h, o)


@pytest.mark.gpu
@pytest.mark.parametrize("time", [0.0, 2500.0])
def test_splat_shaders_match_oracle(hip_ext, time):
    scene, cam = shader_scene(P=4000, seed=12)
    tex = golden_textures()
    rng = np.random.default_rng(7 + int(time))
    ids = rng.integers(0, 10, scene.P)
    texm = _gpu_textures(hip_ext, tex)
    h = hip_forward(hip_ext, scene, cam, time=time, texture_manager=texm, splat_manager=_manager(hip_ext, 1, ids))
    T = {k: oracle.Texture(v, mode=4) for k, v in tex.items()}
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations, splat_shaders=ids, textures=T, error_texture=T["Error"],
                                 time=time)
    _check(h, o)
    # the backward reads the shaded opacities (geomState.conic_opacity after RunSplatShaders)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 21)
    gh = hip_backward(hip_ext, h, dc, do, dd, df)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    for k in ["dL_dopacity", "dL_dmeans2D", "dL_dfeatures", "dL_dcolors"]:
        tol = 2e-5 * max(float(np.abs(go[k]).max()), 1e-12)
        assert_close(k, gh[k], go[k], tol, 2e-3)


@pytest.mark.gpu
def test_missing_texture_uses_error_texture(hip_ext):
    """TextureManager::GetTexture (texture.cu:298-314): an unknown name samples the error texture."""
    scene, cam = shader_scene(P=2000, seed=13)
    tex = golden_textures()
    ids = np.full(scene.P, oracle.SP_DISSOLVE)
    only_err = {"Error": tex["Error"]}
    texm = _gpu_textures(hip_ext, only_err)
    h = hip_forward(hip_ext, scene, cam, time=1500.0, texture_manager=texm, splat_manager=_manager(hip_ext, 1, ids))
    E = oracle.Texture(tex["Error"], mode=4)
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations, splat_shaders=ids, textures={}, error_texture=E,
                                 time=1500.0)
    _check(h, o)


@pytest.mark.gpu
def test_shader_validation_is_loud(hip_ext):
    scene, cam = shader_scene(P=500, seed=14)
    ids = np.full(scene.P, oracle.SP_DISSOLVE)
    with pytest.raises(RuntimeError, match="texture"):       # a textured shader without a manager
        hip_forward(hip_ext, scene, cam, splat_manager=_manager(hip_ext, 1, ids))
    ids = np.full(scene.P, oracle.SP_WIREFRAME)
    with pytest.raises(RuntimeError, match="21"):            # addresses features 6..8 with S = 11
        hip_forward(hip_ext, scene, cam, S=11, splat_manager=_manager(hip_ext, 1, ids))


@pytest.mark.gpu
@pytest.mark.parametrize("S", [21, 11])
def test_partial_shader_sets_match_oracle(hip_ext, S):
    """Only the inputs an active shader writes get working copies, and the pre-shader intermediate
    pass runs only when a depth-reading splat shader (Crack, CrackNoRecon) is active
    (rasterizer.hip); without it, at S <= 12, the shader blend sorts its tiles itself (fused, as the
    default blend). SH CullHalf + default with splat Wireframe / QuantizeLight + default (S = 21),
    or Dissolve / Stencil + default (S = 11, no 21-channel feature views): every output still
    matches the oracle (which copies everything and always runs the pass), and so do the keys and
    the sort order."""
    scene, cam = shader_scene(P=4000, seed=15)
    tex = golden_textures()
    rng = np.random.default_rng(3)
    sh_ids = rng.choice([oracle.SH_NAMES.index("CullHalf"), oracle.SH_NAMES.index("ShDefault")], scene.P)
    sp_set = [oracle.SP_WIREFRAME, oracle.SP_QUANTIZELIGHT] if S == 21 else [oracle.SP_DISSOLVE, oracle.SP_STENCIL]
    sp_ids = rng.choice(sp_set + [oracle.SP_DEFAULT], scene.P)
    texm = _gpu_textures(hip_ext, tex)
    h = hip_forward(hip_ext, scene, cam, S=S, time=700.0, texture_manager=texm,
                    sh_manager=_manager(hip_ext, 0, sh_ids), splat_manager=_manager(hip_ext, 1, sp_ids))
    T = {k: oracle.Texture(v, mode=4) for k, v in tex.items()}
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features[:, :S], sh=scene.sh,
                                 scales=scene.scales, rotations=scene.rotations, sh_shaders=sh_ids,
                                 splat_shaders=sp_ids, textures=T, error_texture=T["Error"], time=700.0)
    _check(h, o)
    import relightable3dgaussian_amd as r

    st = r._C.rasterizer_state(h["geom"], h["binning"], h["image"], scene.P, cam.height, cam.width,
                               h["num_rendered"])
    np.testing.assert_array_equal(st[1].cpu().numpy().view(np.uint32), o["point_list"])
