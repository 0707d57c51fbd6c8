"""Post-process passes: the oracle's literal restatement of
RunPostProcessShaders (forward.cu:973-1047; postProcessShader.cu:177-374; shaderUtils.cu) on the
CPU, and the HIP passes (fused pixel-local launches, snapshot-only BlurLighting) against it on
the GPU.

The reference maps thread idx to pixel (idx % W, idx / H) (postProcessShader.cu:443-444), which
is the pixel grid only for square images (W > H writes out of bounds, W < H races): both sides
use (idx % W, idx / W), and the parity cases include square images, where that is exactly the
reference's mapping. Tolerance: 1e-4 abs (north_star). The passes threshold their inputs
(Sobel's int truncation, roundf quantisation, stencil tests), so a pixel whose input sits
within float rounding of a threshold may legitimately flip: at most 0.1% of the pixels may
differ, and only those.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from tests._helpers import hip_forward
from tests.test_shaders import _gpu_textures, _manager, golden_textures, shader_scene

IMG_ATOL = 1e-4
PP = oracle


def _render(scene, cam, T, passes, splat_ids=None, time=0.0):
    return oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh,
                                    scales=scene.scales, rotations=scene.rotations, splat_shaders=splat_ids,
                                    textures=T, error_texture=T["Error"], time=time, post_passes=passes)


def _stencil_ids(P, seed=0):
    """splat shaders that write stencils / metallic, so the stencil-gated passes do work"""
    rng = np.random.default_rng(seed)
    return rng.choice([oracle.SP_STENCIL, oracle.SP_CRACKNORECON, oracle.SP_DEFAULT], size=P, p=[0.5, 0.3, 0.2])


@pytest.fixture(scope="module")
def tex():
    return {k: oracle.Texture(v, mode=4) for k, v in golden_textures().items()}


def test_default_pass_only_rerenders_depth_and_stencil(tex):
    scene, cam = shader_scene(P=1500, seed=1, width=64, height=64)
    a = _render(scene, cam, tex, None)
    b = _render(scene, cam, tex, [PP.PP_DEFAULT])
    for k in ["color", "opacity", "feature", "shader_color", "normal", "surface_xyz"]:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert np.abs(a["depth"] - b["depth"]).max() > 0       # the intermediate depth replaces the blend's


def test_invert_and_quantize(tex):
    scene, cam = shader_scene(P=1500, seed=2, width=64, height=64)
    a = _render(scene, cam, tex, None)
    b = _render(scene, cam, tex, [PP.PP_INVERT, PP.PP_QUANTIZELIGHTING])
    np.testing.assert_array_equal(b["shader_color"], np.float32(1) - a["shader_color"])
    HW = 64 * 64
    inc_a = a["feature"].reshape(-1)[12 * HW:15 * HW].reshape(HW, 3)
    inc_b = b["feature"].reshape(-1)[12 * HW:15 * HW].reshape(HW, 3)
    q = np.round(inc_a.max(1) * np.float32(4)) / np.float32(4)
    np.testing.assert_array_equal(inc_b, np.repeat(q[:, None], 3, 1))
    rest = np.ones(21 * HW, bool)
    rest[12 * HW:15 * HW] = False
    np.testing.assert_array_equal(b["feature"].reshape(-1)[rest], a["feature"].reshape(-1)[rest])


def test_blur_matches_numpy(tex):
    scene, cam = shader_scene(P=1500, seed=3, width=48, height=40)
    W, H = cam.width, cam.height
    HW = W * H
    a = _render(scene, cam, tex, None)
    b = _render(scene, cam, tex, [PP.PP_BLURLIGHTING])
    inc = a["feature"].reshape(-1)[12 * HW:15 * HW].reshape(HW, 3)
    K = np.array([[0.009375, 0.01875, 0.028125, 0.01875, 0.009375], [0.01875, 0.0375, 0.045, 0.0375, 0.01875],
                  [0.028125, 0.045, 0.3, 0.045, 0.028125], [0.01875, 0.0375, 0.045, 0.0375, 0.01875],
                  [0.009375, 0.01875, 0.028125, 0.01875, 0.009375]], np.float32)
    want = inc.copy()
    for p in range(HW):
        if not inc[p].any():
            continue
        acc = np.zeros(3, np.float32)
        for dx in range(-2, 3):
            for dy in range(-2, 3):
                acc = acc + K[dx + 2, dy + 2] * inc[min(max(p + dx + dy * W, 0), HW - 1)]
        want[p] = acc
    got = b["feature"].reshape(-1)[12 * HW:15 * HW].reshape(HW, 3)
    np.testing.assert_array_equal(got, want)


def test_outline_copies_base_colour(tex):
    """OutlineShader samples in.pixel itself (postProcessShader.cu:224), so no pixel is outlined
    and the pass writes the base colour."""
    scene, cam = shader_scene(P=1500, seed=4, width=64, height=64)
    b = _render(scene, cam, tex, [PP.PP_OUTLINE], splat_ids=_stencil_ids(scene.P))
    HW = 64 * 64
    base = b["feature"].reshape(-1)[9 * HW:12 * HW].reshape(64, 64, 3)
    np.testing.assert_array_equal(b["shader_color"], base)


def test_stencil_gated_passes_do_work(tex):
    scene, cam = shader_scene(P=2500, seed=5, width=64, height=64)
    ids = _stencil_ids(scene.P, 5)
    a = _render(scene, cam, tex, [PP.PP_DEFAULT], splat_ids=ids)
    assert (a["stencil"] > 0.01).mean() > 0.2
    for passes in ([PP.PP_TEXTUREDSHADOWS], [PP.PP_CRACKRECON], [PP.PP_TOON]):
        b = _render(scene, cam, tex, passes, splat_ids=ids)
        assert np.abs(b["shader_color"] - a["shader_color"]).max() > 0.05, passes


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
CASES = [
    ([PP.PP_TOON], 64, 64),
    ([PP.PP_CRACKRECON, PP.PP_INVERT, PP.PP_SOBEL], 80, 80),
    ([PP.PP_QUANTIZELIGHTING, PP.PP_BLURLIGHTING, PP.PP_TEXTUREDSHADOWS, PP.PP_BLURLIGHTING], 64, 64),
    ([PP.PP_OUTLINE, PP.PP_DEFAULT, PP.PP_SOBEL, PP.PP_INVERT], 96, 72),   # non-square: the intended mapping
]


def _check_images(h, o):
    for k in ["color", "opacity", "depth", "stencil", "normal", "surface_xyz"]:
        d = np.abs(h[k].cpu().numpy().astype(np.float64) - o[k])
        assert d.max() <= IMG_ATOL, f"{k}: max abs diff {d.max():.3e}"
    for k, hv, ov in [("shader_color", h["shader_color"].cpu().numpy(), o["shader_color"]),
                      ("feature", h["feature"].cpu().numpy().reshape(-1), o["feature"].reshape(-1))]:
        d = np.abs(hv.astype(np.float64) - ov)
        frac = float((d > IMG_ATOL).mean())
        assert frac <= 1e-3, f"{k}: {frac:.2e} of the values off (max {d.max():.3e})"


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)))
def test_post_passes_match_oracle(hip_ext, case):
    passes, W, H = CASES[case]
    scene, cam = shader_scene(P=4000, seed=20 + case, width=W, height=H)
    texs = golden_textures()
    T = {k: oracle.Texture(v, mode=4) for k, v in texs.items()}
    ids = _stencil_ids(scene.P, case)
    texm = _gpu_textures(hip_ext, texs)
    pmap = hip_ext.GetPostProcessShaderAddressMap()
    handles = [pmap[oracle.POST_NAMES[i]] for i in passes]
    h = hip_forward(hip_ext, scene, cam, texture_manager=texm, splat_manager=_manager(hip_ext, 1, ids),
                    post_passes=handles)
    o = _render(scene, cam, T, passes, splat_ids=ids)
    _check_images(h, o)


@pytest.mark.gpu
def test_post_pass_validation_is_loud(hip_ext):
    scene, cam = shader_scene(P=500, seed=30, width=32, height=32)
    pmap = hip_ext.GetPostProcessShaderAddressMap()
    with pytest.raises(RuntimeError, match="21"):          # reads the 21-channel feature image
        hip_forward(hip_ext, scene, cam, S=11, post_passes=[pmap["QuantizeLighting"]])
    with pytest.raises(RuntimeError, match="shadow"):      # samples "shadow" without a texture manager
        hip_forward(hip_ext, scene, cam, post_passes=[pmap["ToonShader"]])
    with pytest.raises(RuntimeError, match="handle"):
        hip_forward(hip_ext, scene, cam, post_passes=[12345])
    # S != 21 is fine for passes that do not read features
    hip_forward(hip_ext, scene, cam, S=11, post_passes=[pmap["Invert"], pmap["SobelFilter"]])
