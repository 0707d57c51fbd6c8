"""Call-site replay of gaussian_renderer/neilf.py through the shipped
wrapper (relightable3dgaussian_amd.r3dg_rasterization: GaussianRasterizer, RenderEquation,
RenderEquation_complex), checked against the oracle.

The sequences are written out here in this test's own code, following the reference's steps:
  eval (neilf.py:96-170):   complex BRDF -> per-sample .mean(-2) -> 21-channel torch.cat ->
                            rasterizer -> .reshape(-1).view(21,H,W).split([1,1,1,3,3,3,3,3,3], 0)
                            -> each block .view(H,W,n) -> pbr + (1 - opacity) * bg;
  training (neilf.py:96-147): training BRDF (random rotation) -> 11-channel cat -> rasterizer ->
                            the split of integration/neilf_training_split.patch (the reference's
                            own line, split along dim=2, raises for any layout) -> loss -> backward
                            through the rasterizer and the BRDF.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from relightable3dgaussian_amd import synthetic
from tests._helpers import assert_close, upstream_grads

pytestmark = pytest.mark.gpu

EVAL_GROUPS = [1, 1, 1, 3, 3, 3, 3, 3, 3]  # neilf.py:150
EVAL_NAMES = ["roughness", "metallic", "visibility", "pbr", "normal", "base_color", "lights", "local_lights",
              "global_lights"]
TRAIN_GROUPS = [1, 1, 3, 3, 3]  # neilf.py:142
TRAIN_NAMES = ["roughness", "metallic", "pbr", "normal", "base_color"]


def _inputs(seed, P=3000, width=96, height=72):
    scene, cam = synthetic.small_scene(P=P, S=1, seed=seed, width=width, height=height)
    b = synthetic.brdf_inputs(P, seed=seed + 1, S=16)
    v = cam.campos[None, :] - scene.means3D  # neilf.py:103 viewdirs = normalize(camera_center - means3D)
    b["viewdirs"] = (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)
    return scene, cam, b


def _planar(o, S, HW):
    """The oracle's feature buffer as planar channels [S, HW] (its layout statement, forward.cu:537-558)."""
    fa, fm = oracle.feature_layout(S, HW)
    flat = o["feature"].reshape(-1)
    return np.stack([flat[fa[c] + np.arange(HW) * fm[c]] for c in range(S)])


def _rasterizer(cam, bg):
    from relightable3dgaussian_amd.r3dg_rasterization import GaussianRasterizer, settings_from_camera

    return GaussianRasterizer(settings_from_camera(cam, bg))


def test_neilf_eval_sequence(hip_ext):
    import torch

    from relightable3dgaussian_amd.r3dg_rasterization import RenderEquation_complex

    scene, cam, b = _inputs(seed=50)
    H, W = cam.height, cam.width
    bg = (0.2, 0.4, 0.6)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda")  # noqa: E731
    base, rough, metal, normal = t(b["base"]), t(b["rough"]), t(b["metal"]), t(b["normals"])
    viewdirs, incidents, env, vis = t(b["viewdirs"]), t(b["incidents"]), t(b["env"]), t(b["visibility"])
    with torch.no_grad():
        (pbr, _, incident_lights, local_incident_lights, global_incident_lights, incident_visibility, diffuse_light,
         local_diffuse_light, accum, rgb_d, rgb_s) = RenderEquation_complex(base, rough, metal, normal, viewdirs,
                                                                             incidents, env, vis, sample_num=24)
        features = torch.cat([rough, metal, incident_visibility.mean(-2), pbr, normal, base,
                              incident_lights.mean(-2), local_incident_lights.mean(-2),
                              global_incident_lights.mean(-2)], dim=-1)
        assert features.shape == (scene.P, 21)
        means3D = t(scene.means3D)
        out = _rasterizer(cam, bg)(means3D=means3D, means2D=torch.zeros_like(means3D), shs=t(scene.sh),
                                   colors_precomp=None, opacities=t(scene.opacity), scales=t(scene.scales),
                                   rotations=t(scene.rotations), cov3D_precomp=None, features=features)
    (num_rendered, num_contrib, rendered_image, rendered_opacity, rendered_depth, rendered_stencil, rendered_feature,
     rendered_shader, rendered_pseudo_normal, rendered_surface_xyz, radii) = out
    blocks = list(rendered_feature.reshape(-1).view(21, H, W).split(EVAL_GROUPS, dim=0))
    blocks = [f.view(H, W, f.shape[0]) for f in blocks]
    bgt = torch.tensor(bg, device="cuda")
    composite = blocks[3] + (1 - rendered_opacity) * bgt[None, None, :]

    # oracle: the same sequence on the CPU restatements
    ob = oracle.brdf_forward_complex(b, 24)
    ofeat = np.concatenate([b["rough"], b["metal"], ob["incident_visibility"].mean(-2), ob["pbr"], b["normals"],
                            b["base"], ob["incident_lights"].mean(-2), ob["local_incident_lights"].mean(-2),
                            ob["global_incident_lights"].mean(-2)], axis=-1).astype(np.float32)
    assert_close("features", features.cpu().numpy(), ofeat, 2e-5, 1e-4)
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, ofeat, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations, bg=bg)
    assert int(num_rendered) == o["num_rendered"]
    np.testing.assert_array_equal(num_contrib.cpu().numpy(), o["n_contrib"])
    planar = _planar(o, 21, H * W)
    c = 0
    for name, n, blk in zip(EVAL_NAMES, EVAL_GROUPS, blocks):
        ref = planar[c:c + n].T.reshape(H, W, n)
        assert_close(name, blk.cpu().numpy(), ref, 1e-4, 1e-4)
        c += n
    ocomp = planar[3:6].T.reshape(H, W, 3) + (1 - o["opacity"]) * np.asarray(bg, np.float32)[None, None, :]
    assert_close("pbr composite", composite.cpu().numpy(), ocomp, 1e-4, 1e-4)
    assert_close("render", rendered_image.cpu().numpy(), o["color"], 1e-4)


def test_neilf_training_sequence(hip_ext):
    import torch

    from relightable3dgaussian_amd.r3dg_rasterization import RenderEquation

    scene, cam, b = _inputs(seed=60)
    H, W = cam.height, cam.width
    bg = (1.0, 1.0, 1.0)
    leaf = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
    base, rough, metal, normal = leaf(b["base"]), leaf(b["rough"]), leaf(b["metal"]), leaf(b["normals"])
    incidents, env, vis = leaf(b["incidents"]), leaf(b["env"]), leaf(b["visibility"])
    means3D, opac, sh = leaf(scene.means3D), leaf(scene.opacity), leaf(scene.sh)
    scales, rots = leaf(scene.scales), leaf(scene.rotations)
    viewdirs = torch.nn.functional.normalize(torch.tensor(cam.campos, device="cuda") - means3D, dim=-1)
    brdf_color, incident_dirs, diffuse_light = RenderEquation(base, rough, metal, normal.detach(), viewdirs, incidents,
                                                              env, vis, 24, True)
    features = torch.cat([rough, metal, brdf_color, normal, base], dim=-1)
    features.retain_grad()
    means2D = torch.zeros_like(means3D, requires_grad=True)
    out = _rasterizer(cam, bg)(means3D=means3D, means2D=means2D, shs=sh, colors_precomp=None, opacities=opac,
                               scales=scales, rotations=rots, cov3D_precomp=None, features=features)
    rendered_image, rendered_opacity, rendered_feature = out[2], out[3], out[6]
    with pytest.raises(RuntimeError):  # the reference's own line (neilf.py:142), at this image's size
        rendered_feature.reshape(-1).view(11, H, W).split(TRAIN_GROUPS, dim=2)
    blocks = [f.view(H, W, f.shape[0]) for f in  # integration/neilf_training_split.patch
              rendered_feature.reshape(-1).view(11, H, W).split(TRAIN_GROUPS, dim=0)]
    rendered_roughness, rendered_metallic, rendered_pbr, rendered_normal, rendered_base_color = blocks

    # the oracle renders the same per-Gaussian features (the training BRDF draws its own rotation)
    fin = features.detach().cpu().numpy()
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, fin, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations, bg=bg)
    planar = _planar(o, 11, H * W)
    c = 0
    for name, n, blk in zip(TRAIN_NAMES, TRAIN_GROUPS, blocks):
        assert_close(name, blk.detach().cpu().numpy(), planar[c:c + n].T.reshape(H, W, n), 1e-4, 1e-4)
        c += n

    # loss over the split views + the image; gradients reach the features through the rasterizer
    dc, _, _, df = upstream_grads(H, W, 11, seed=8)
    g = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda")  # noqa: E731
    loss = (rendered_image * g(dc.transpose(1, 2, 0))).sum()
    c = 0
    for n, blk in zip(TRAIN_GROUPS, blocks):
        loss = loss + (blk * g(df[c:c + n].reshape(n, H * W).T.reshape(H, W, n))).sum()
        c += n
    loss.backward()
    zero = np.zeros(H * W, np.float32)
    go = oracle.rasterize_backward(o, dc, zero, zero, df)
    ref = go["dL_dfeatures"]
    assert_close("features.grad", features.grad.cpu().numpy(), ref, 2e-5 * float(np.abs(ref).max()), 2e-3)
    for name, p in [("base", base), ("rough", rough), ("metal", metal), ("incidents", incidents), ("env", env),
                    ("visibility", vis), ("opacity", opac), ("sh", sh), ("scales", scales)]:
        gr = p.grad
        assert gr is not None and bool(torch.isfinite(gr).all()), name
        assert float(gr.abs().max()) > 0, name
    # base_color reaches the loss twice: directly (feature channels 8..10) and through the BRDF
    direct = features.grad[:, 8:11]
    assert float((base.grad - direct).abs().max()) > 0
