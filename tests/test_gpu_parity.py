"""GPU parity: the HIP path (through the _C boundary) against the CPU oracle.

Tolerances (north_star, BASELINE.json): rendered images / features within 1e-4 abs fp32; tile
keys, sort order (point list), tile ranges, radii and num_rendered bit-exact. Gradients have no
stated tolerance; they are compared at rtol 2e-3 + 2e-5 * max|ref| (summation order differs:
the HIP backward reduces per wave and per Gaussian row, the oracle sums pixel by pixel).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
from relightable3dgaussian_amd import synthetic
from tests._helpers import (assert_brdf, assert_close, check_grad, hip_backward, hip_forward, lib_options,
                            rows_reduction, tt, upstream_grads)

pytestmark = pytest.mark.gpu

IMG_ATOL = 1e-4


def _oracle_fwd(scene, cam, S, use_cov=False, colors=None, degree=3, bg=(1.0, 1.0, 1.0), scale_modifier=1.0):
    cov = oracle.cov3d(scene.scales, scene.rotations, scale_modifier) if use_cov else None
    return oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features[:, :S],
                                    sh=None if colors is not None else scene.sh, degree=degree,
                                    scales=None if use_cov else scene.scales,
                                    rotations=None if use_cov else scene.rotations, cov3D_precomp=cov,
                                    colors_precomp=colors, bg=bg, scale_modifier=scale_modifier)


def _final_T(h, cam):
    import torch

    HW = cam.height * cam.width
    return h["image"][: HW * 4].view(torch.float32).cpu().numpy()  # image state starts with final_T


def _check_forward(h, o, S):
    import relightable3dgaussian_amd as r

    assert h["num_rendered"] == o["num_rendered"]
    P = o["radii"].shape[0]
    cam = h["_cam"]
    L = h["num_rendered"]
    st = r._C.rasterizer_state(h["geom"], h["binning"], h["image"], P, cam.height, cam.width, L)
    keys, plist, ranges = (t.cpu().numpy() for t in st[:3])
    np.testing.assert_array_equal(keys.view(np.uint64), o["keys"])           # tile|depth keys
    np.testing.assert_array_equal(plist.view(np.uint32), o["point_list"])    # sort order
    np.testing.assert_array_equal(ranges.view(np.uint32), o["ranges"])       # tile ranges
    np.testing.assert_array_equal(h["radii"].cpu().numpy(), o["radii"])
    vis = o["radii"] > 0
    np.testing.assert_array_equal(st[4].cpu().numpy()[vis], o["depths"][vis])
    for k in ["color", "opacity", "depth", "shader_color"]:
        assert_close(k, h[k].cpu().numpy(), o[k], IMG_ATOL)
    assert_close("feature", h["feature"].cpu().numpy().reshape(-1), o["feature"].reshape(-1), IMG_ATOL)
    # alpha, T and the early stop are bit-identical (gauss_power + r3dg_expf on both sides)
    np.testing.assert_array_equal(h["n_contrib"].cpu().numpy(), o["n_contrib"])
    np.testing.assert_array_equal(_final_T(h, cam), o["final_T"])
    np.testing.assert_array_equal(h["stencil"].cpu().numpy(), 0.0)


@pytest.mark.parametrize("S", [0, 3, 6, 11, 12, 16, 21, 32])  # every SMAX instantiation (S <= 0/4/8/11/12/16/24/32)
def test_forward_matches_oracle(hip_ext, S):
    scene, cam = synthetic.small_scene(P=3000, S=max(S, 21), seed=S, width=96, height=72)
    h = hip_forward(hip_ext, scene, cam, S=S)
    o = _oracle_fwd(scene, cam, S)
    _check_forward(h, o, S)


def test_forward_pseudo_normal_and_xyz(hip_ext):
    scene, cam = synthetic.small_scene(P=4000, S=11, seed=7, width=80, height=64)
    h = hip_forward(hip_ext, scene, cam, S=11)
    o = _oracle_fwd(scene, cam, 11)
    op = o["opacity"][..., 0]
    # where the surface is defined (opacity well above 0 in the 3x3 neighbourhood) the xyz /
    # normal buffers follow the 1e-4 image tolerance; depth / max(opacity, 1e-7) amplifies
    # last-bit differences where the opacity is ~0, so those pixels get a relative bound
    from scipy.ndimage import minimum_filter

    solid = minimum_filter(op, size=3, mode="nearest") > 0.2
    hx, ox = h["surface_xyz"].cpu().numpy(), o["surface_xyz"]
    assert_close("surface_xyz", hx[solid], ox[solid], 1e-4, 1e-5)
    assert_close("surface_xyz(all)", hx, ox, 1e-3, 1e-3)
    hn, on = h["normal"].cpu().numpy(), o["normal"]
    assert_close("normal", hn[solid], on[solid], 1e-4, 1e-4)


def test_dense_tiles_depth_sort(hip_ext):
    """Tiles longer than one depth-sort chunk (preprocess.hip tile_depth_sort_kernel: tiles of up
    to 1024 instances sort in one 1024-chunk, longer ones in 2048-instance chunks whose sorted runs
    merge in ceil(log2(chunks)) ping-pong rounds) with many exact depth ties (the reference orders
    ties by Gaussian id). The density falls off across a 96x48 frame so the tiles span 0, 1, 2 and
    3 merge rounds -- both parities of the ping-pong: keys, point list and ranges bit-exact, images
    within 1e-4, gradients at the usual bar."""
    import math

    P = 60000
    scene, cam = synthetic.small_scene(P=P, S=11, seed=40, width=96, height=48, scale_range=(0.02, 0.12))
    m = scene.means3D.copy()
    u = np.random.default_rng(41).uniform(0, 1, P) ** 3.0  # dense near the left edge
    m[:, 0] = (u * 2 - 1) * m[:, 2] * math.tan(cam.fovx / 2) * 1.2
    m[:, 2] = np.round(m[:, 2] * 4.0) / 4.0  # 15 distinct depths: thousands of ties per tile
    m[:, :2] *= (m[:, 2] / scene.means3D[:, 2])[:, None]
    scene = synthetic.Scene(m, scene.scales, scene.rotations, scene.opacity, scene.sh, scene.features)
    h = hip_forward(hip_ext, scene, cam, S=11)
    o = _oracle_fwd(scene, cam, 11)
    counts = o["ranges"][:, 1].astype(np.int64) - o["ranges"][:, 0]
    rounds = np.ceil(np.log2(np.maximum(np.ceil(counts / 2048), 1))).astype(int)
    long = counts > 1024
    assert set(rounds[long].tolist()) >= {0, 1, 2, 3}, sorted(counts.tolist())
    _check_forward(h, o, 11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=6)
    gh = hip_backward(hip_ext, h, dc, do, dd, df)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    grad_check("dense_tiles", gh, go, ["dL_dmeans2D", "dL_dopacity", "dL_dfeatures", "dL_dmeans3D", "dL_dsh"])


def test_cull_is_exact(hip_ext):
    """The per-quadrant footprint skip must not change a single bit (render_fwd.hip): forward and
    rows-reduction backward bitwise, the default atomic backward within assert_hip_runs_agree."""
    scene, cam = synthetic.small_scene(P=5000, S=11, seed=3, width=128, height=96, scale_range=(0.005, 0.3))
    _cull_on_off(hip_ext, scene, cam)


def assert_hip_runs_agree(tag, ga, gb, keys=None):
    """Two HIP backward runs on the default atomic flush (order-dependent last bits: a different
    f32 summation order, like the oracle's own): within GRAD_BARS of each other."""
    for k in keys or ga:
        rel, frac = GRAD_BARS.get(k, (1e-4, 2e-5))
        m = max(float(np.abs(gb[k]).max()) if gb[k].size else 0.0, 1e-12)
        assert_close(f"{tag} {k}", ga[k], gb[k], frac * m, rel)


def _cull_on_off(hip_ext, scene, cam, S=11, seed=1, atomic_keys=None):
    """Cull on == cull off: forward bitwise; the backward bitwise on the deterministic rows
    reduction, and on the default atomic flush within assert_hip_runs_agree (over atomic_keys: the
    well-conditioned gradients; the caller checks the others). Returns the forward, the default
    (atomic) gradients of both runs and the upstream gradients."""
    a = hip_forward(hip_ext, scene, cam, S=S)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, S, seed=seed)
    with rows_reduction():  # the two backward runs are compared bit for bit
        ga = hip_backward(hip_ext, a, dc, do, dd, df)
    ga_atomic = hip_backward(hip_ext, a, dc, do, dd, df)
    with lib_options(test_no_cull=1):
        b = hip_forward(hip_ext, scene, cam, S=S)
        with rows_reduction():
            gb = hip_backward(hip_ext, b, dc, do, dd, df)
        gb_atomic = hip_backward(hip_ext, b, dc, do, dd, df)
    for k in ["color", "opacity", "depth", "feature", "n_contrib", "normal", "surface_xyz"]:
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)
    for k in ga:
        np.testing.assert_array_equal(ga[k], gb[k], err_msg=k)
    assert_hip_runs_agree("cull on/off atomic", ga_atomic, gb_atomic, atomic_keys)
    return a, (ga_atomic, gb_atomic, ga), (dc, do, dd, df)


@pytest.mark.timeout(400)
def test_cull_exact_needles(hip_ext):
    """The quadrant cull where fp32 rounding is largest (r3dg_common.h rect_culled): 1920x1080,
    300 faint needles (sigma 100-1000 px along a screen diagonal, the 0.3 px^2 low-pass floor
    across, opacity 0.005-0.05, means mostly far outside the tiles they cover). The conic form's
    terms reach ~1e6 and cancel to a few units there. Cull on == off bit for bit (forward and
    backward); keys, n_contrib and final_T bit-exact against the oracle, images within 1e-4, the
    well-conditioned gradients against the oracle, the ill-conditioned ones within the oracle's own
    fp32 rounding sensitivity (see the comments)."""
    cam = synthetic.m1_camera()
    scene = synthetic.needle_scene(300, S=11, seed=0, cam=cam)
    well = ["dL_dcolors", "dL_dopacity", "dL_dfeatures"]
    h, (gh, gh_off, g_rows), (dc, do, dd, df) = _cull_on_off(hip_ext, scene, cam, atomic_keys=well)
    o = _oracle_fwd(scene, cam, 11)
    assert o["num_rendered"] > 1_000_000 and int(o["n_contrib"].max()) > 100
    _check_forward(h, o, 11)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    grad_check("needles", gh, go, well)
    # the default atomic flush, cull on AND off, each against the oracle at the conditioning bounds
    # below (cull on / off with the deterministic rows reduction are bitwise equal, _cull_on_off)
    # the atomic flush's summation order is one more perturbation of these sums: the spread among
    # three summation orders of the same rows (two atomic runs with different arrival orders and the
    # rows reduction's fixed order) joins the ulp spread
    order = {}
    for k in ["dL_dmeans3D", "dL_dcov3D", "dL_dscales", "dL_drotations"]:
        runs = [x[k].astype(np.float64).reshape(x[k].shape[0], -1) for x in (gh, gh_off, g_rows)]
        order[k] = np.max([np.abs(p - q).max(1) for i, p in enumerate(runs) for q in runs[i + 1:]], axis=0)
    go64 = oracle.rasterize_backward(o, dc, do, dd, df, acc64=True)
    _needle_ill_conditioned([gh, gh_off, g_rows], go, o, dc, do, dd, df, order, go64)


def _needle_ill_conditioned(ghs, go, o, dc, do, dd, df, order=None, go64=None):
    # dL/dmean2D = -0.5 W o (a Sdx + b Sdy): for a diagonal needle a ~ -b and Sdx ~ Sdy (pixel
    # offsets of ~1e3 px), so the product cancels by ~1e3 and two fp32 summation orders of the pixel
    # terms (the reference's own atomics included) differ there at ~2e-4 of the largest gradient
    # (measured 2.3e-4): bar 1e-3 of the maximum.
    for gh in ghs:
        err = float(np.abs(gh["dL_dmeans2D"].astype(np.float64) - go["dL_dmeans2D"]).max())
        print(f"needles dL_dmeans2D: max |diff| / max |ref| = {err / float(np.abs(go['dL_dmeans2D']).max()):.2e}")
        assert_close("dL_dmeans2D", gh["dL_dmeans2D"], go["dL_dmeans2D"],
                     1e-3 * float(np.abs(go["dL_dmeans2D"]).max()), 2e-3)
    # dL/dcov3D and the cov2D part of dL/dmeans3D go through the conic inverse (backward.cu:
    # 180-230): with cov2D ~ [[5e5, +-5e5], [+-5e5, 5e5]] its determinant is a ~1e6-fold cancellation
    # of a*c against b^2 in fp32, so an fp32 rounding of dL/dconic moves them by O(1). Their bar is
    # the problem's own sensitivity: the oracle run again on upstream gradients moved by one ulp
    # each (random direction, four draws) spreads by s per Gaussian -- a lower estimate of the
    # sensitivity, four draws of many -- and the GPU's summation order is one more such draw: it
    # must lie within 16 * max(s) of the oracle per Gaussian (+ 2e-5 of the largest gradient); s
    # also takes the spread between the GPU's summation orders, and the f32 oracle's own error: its
    # per-pixel terms are themselves ~1e3-fold cancellations (dG/ddelx = -G dx a - G dy b on a
    # diagonal needle) summed in f32, so it sits off the exact sum of its own per-pixel values (the
    # acc64 oracle: same f32 per-pixel chain, terms and sums in double) by e per Gaussian. The GPU
    # sums moments in double, so it is held to the acc64 oracle at the same bound.
    # (Measured round 4, rows reduction in f32: worst GPU diff / (4 * spread) = 8 on one Gaussian of
    # 300; round 5, moments in double: 1.7x the ulp-only 16x bound on one Gaussian, from the f32
    # oracle's own error.)
    rng = np.random.default_rng(99)
    spread = {k: np.zeros(go[k].shape[0]) for k in ["dL_dmeans3D", "dL_dcov3D", "dL_dscales", "dL_drotations"]}
    for _ in range(4):
        pert = [np.nextafter(x, np.where(rng.random(x.shape) < 0.5, -np.inf, np.inf).astype(np.float32))
                .astype(np.float32) for x in (dc, do, dd, df)]
        gp = oracle.rasterize_backward(o, *pert)
        for k in spread:
            d = np.abs(gp[k].astype(np.float64) - go[k]).reshape(go[k].shape[0], -1).max(1)
            spread[k] = np.maximum(spread[k], d)
    for gh in ghs:
        for k, s in spread.items():
            assert np.isfinite(gh[k]).all(), k
            diff = np.abs(gh[k].astype(np.float64) - go[k]).reshape(go[k].shape[0], -1).max(1)
            sk = np.maximum(s, order[k]) if order is not None else s
            e = np.zeros_like(sk)
            if go64 is not None:
                e = np.abs(go[k].astype(np.float64) - go64[k]).reshape(go[k].shape[0], -1).max(1)
                sk = np.maximum(sk, e)
            bound = 16.0 * sk + 2e-5 * float(np.abs(go[k]).max())
            print(f"needles {k}: max diff {diff.max():.3e}, oracle rounding spread up to {s.max():.3e}, "
                  f"GPU order spread up to {order[k].max() if order is not None else 0:.3e}, "
                  f"f32 oracle off its acc64 sums up to {e.max():.3e}, worst diff/bound {float((diff / bound).max()):.3f}")
            assert np.all(diff <= bound), (k, int((diff > bound).sum()), float((diff / bound).max()))
            if go64 is not None:
                d64 = np.abs(gh[k].astype(np.float64) - go64[k]).reshape(go[k].shape[0], -1).max(1)
                print(f"needles {k}: GPU off the acc64 oracle up to {d64.max():.3e} "
                      f"(f32 oracle {e.max():.3e}), worst / bound {float((d64 / bound).max()):.3f}")
                assert np.all(d64 <= bound), (k, "acc64", float((d64 / bound).max()))


@rows_reduction()  # the feature gradients of two backward runs are compared bit for bit
def test_backward_geometry_false(hip_ext):
    """backward_geometry=False drops the feature term of dL/dalpha (backward.cu:563): matches the
    oracle run the same way, and differs from the default where features carry gradient."""
    scene, cam = synthetic.small_scene(P=2500, S=11, seed=17, width=96, height=64)
    h = hip_forward(hip_ext, scene, cam, S=11)
    o = _oracle_fwd(scene, cam, 11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=5)
    df = df * 100.0  # feature grads dominate dL/dalpha, so dropping them is visible
    gh = hip_backward(hip_ext, h, dc, do, dd, df, backward_geometry=False)
    go = oracle.rasterize_backward(o, dc, do, dd, df, backward_geometry=False)
    grad_check("bwd_geometry_false", gh, go)
    gt = hip_backward(hip_ext, h, dc, do, dd, df, backward_geometry=True)
    # the feature gradients themselves do not depend on the flag; the geometry gradients do
    np.testing.assert_array_equal(gt["dL_dfeatures"], gh["dL_dfeatures"])
    assert np.abs(gt["dL_dopacity"] - gh["dL_dopacity"]).max() > 1e-3 * np.abs(gt["dL_dopacity"]).max()


def test_prefiltered(hip_ext):
    """prefiltered=True (auxiliary.h:154-160): a set the caller promises is inside the frustum
    renders exactly as prefiltered=False; a point the near-plane test drops, which the reference
    answers with printf + __trap(), fails the call with a RuntimeError naming the cause."""
    scene, cam = synthetic.small_scene(P=800, S=11, seed=23)
    base = hip_forward(hip_ext, scene, cam, S=11)
    pre = hip_forward(hip_ext, scene, cam, S=11, prefiltered=True)
    for k in ["color", "opacity", "depth", "feature", "n_contrib", "radii"]:
        np.testing.assert_array_equal(pre[k].cpu().numpy(), base[k].cpu().numpy(), err_msg=k)
    m = scene.means3D.copy()
    m[7] = np.asarray(cam.campos, np.float32)  # view depth 0 <= 0.2: dropped by the near plane
    bad = synthetic.Scene(m, scene.scales, scene.rotations, scene.opacity, scene.sh, scene.features)
    with pytest.raises(RuntimeError, match="prefiltered"):
        hip_forward(hip_ext, bad, cam, S=11, prefiltered=True)
    # the device stays usable and the flag is per call
    again = hip_forward(hip_ext, scene, cam, S=11, prefiltered=True)
    np.testing.assert_array_equal(again["color"].cpu().numpy(), base["color"].cpu().numpy())


# Raster-gradient bars against the oracle: |HIP - oracle| <= rel |ref| + frac max|ref| per element
# (tests/_helpers.py check_grad prints the measured max|d|/max|ref| and relative error; DESIGN.md §5
# records them).
# Set at <= ~4x the largest error measured on the default build over M1, C2, C3, C4, the C5 view and
# the small-scene tests (profiles/r05/grad_report.jsonl), with rel = 1e-4 for all. The
# colour / feature / SH gradients carry the two-term bf16 split of w = alpha T (|w - h - m| <=
# 2^-16 |w|): ~7.6e-6 of max|ref| measured (the exact three-term split: ~2e-6, the one-term
# reduction: 3.7e-3 -- test_one_term_reduction_fails_bar); mean2D / opacity / means3D come from the
# exact moment products (<= 2.5e-7 / 6.3e-7 / 4.3e-7 measured). Round 4's bar was 2e-3 |ref| +
# 2e-5 max|ref| for all.
GRAD_BARS = {"dL_dmeans2D": (1e-4, 1e-6), "dL_dopacity": (1e-4, 2.5e-6), "dL_dmeans3D": (1e-4, 1.5e-6),
             "dL_dcolors": (1e-4, 2e-5), "dL_dfeatures": (1e-4, 2e-5), "dL_dsh": (1e-4, 2e-5),
             "dL_dcov3D": (1e-4, 2e-5), "dL_dscales": (1e-4, 2e-5), "dL_drotations": (1e-4, 2e-5)}


def grad_check(tag, gh, go, keys=None):
    for k in keys or GRAD_BARS:
        if k in go and k in gh:
            check_grad(tag, k, gh[k], go[k], *GRAD_BARS[k])


@pytest.mark.parametrize("S", [0, 3, 6, 11, 12, 16, 21, 24, 32])  # every SMAX instantiation
def test_backward_matches_oracle(hip_ext, S):
    scene, cam = synthetic.small_scene(P=2500, S=max(S, 21), seed=10 + S, width=96, height=64)
    h = hip_forward(hip_ext, scene, cam, S=S)
    o = _oracle_fwd(scene, cam, S)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, S)
    gh = hip_backward(hip_ext, h, dc, do, dd, df)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    grad_check(f"bwd S={S}", gh, go)


def test_backward_precomputed_colors_and_cov(hip_ext):
    scene, cam = synthetic.small_scene(P=2000, S=11, seed=21, width=64, height=64)
    colors = np.random.default_rng(5).uniform(0, 1, (scene.P, 3)).astype(np.float32)
    h = hip_forward(hip_ext, scene, cam, S=11, colors=colors, use_cov=True)
    o = _oracle_fwd(scene, cam, 11, use_cov=True, colors=colors)
    _check_forward(h, o, 11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=4)
    gh = hip_backward(hip_ext, h, dc, do, dd, df)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    grad_check("precomputed", gh, go, ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dfeatures", "dL_dmeans3D", "dL_dcov3D"])
    assert np.all(gh["dL_dscales"] == 0) and np.all(gh["dL_drotations"] == 0)


def test_backward_deterministic(hip_ext):
    """The deterministic reduction (bwd_reduce = rows: partial rows summed in a fixed order) gives
    bitwise the same gradients run to run."""
    scene, cam = synthetic.small_scene(P=3000, S=11, seed=2, width=96, height=96)
    with rows_reduction():
        h = hip_forward(hip_ext, scene, cam, S=11)
        dc, do, dd, df = upstream_grads(cam.height, cam.width, 11)
        g1 = hip_backward(hip_ext, h, dc, do, dd, df)
        g2 = hip_backward(hip_ext, h, dc, do, dd, df)
    for k in g1:
        np.testing.assert_array_equal(g1[k], g2[k], err_msg=k)


@pytest.mark.parametrize("size", [(100, 90), (208, 160)])
def test_backward_launch_orders(hip_ext, size):
    """The backward's tile launch order only schedules: longest tiles first (default,
    tile_ranges_kernel; padded-grid slots past the last tile are empty) and the XCD-aware spatial
    order (test_tile_order_spatial) give bitwise the same gradients on the rows reduction. 100 x 90: 42
    tiles on a 48-workgroup grid; 208 x 160: 130 tiles on 136."""
    W, H = size
    scene, cam = synthetic.small_scene(P=3000, S=11, seed=4, width=W, height=H)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11)
    g = {}
    with rows_reduction():
        h = hip_forward(hip_ext, scene, cam, S=11)
        for order in ("longest", "xcd"):
            with lib_options(test_tile_order_spatial=int(order == "xcd")):
                g[order] = hip_backward(hip_ext, h, dc, do, dd, df)
    for k in g["longest"]:
        np.testing.assert_array_equal(g["xcd"][k], g["longest"][k], err_msg=k)


@pytest.mark.parametrize("reduce", ["rows", "atomic"])
def test_backward_ex_layouts(hip_ext, reduce):
    """HWC colour / native feature grads (the wrapper's entry) == CHW / planar (reference contract):
    bitwise on the rows reduction, within assert_hip_runs_agree on the default atomic flush."""
    if reduce == "rows":
        with rows_reduction():
            _ex_layouts(hip_ext, exact=True)
    else:
        _ex_layouts(hip_ext, exact=False)


def _ex_layouts(hip_ext, exact):
    import torch

    import relightable3dgaussian_amd as r
    from tests._helpers import tt

    scene, cam = synthetic.small_scene(P=2000, S=21, seed=8, width=64, height=48)
    h = hip_forward(hip_ext, scene, cam, S=21)
    H, W = cam.height, cam.width
    dc, do, dd, df = upstream_grads(H, W, 21)
    g_ref = hip_backward(hip_ext, h, dc, do, dd, df)
    groups = r._C.feature_groups(21)
    native = np.zeros(H * W * 21, np.float32)
    c = 0
    for n in groups:  # planar [S,H,W] -> forward block layout
        native[H * W * c:H * W * (c + n)] = df[c:c + n].reshape(n, H * W).T.reshape(-1)
        c += n
    a = h["_args"]
    out = r._C.rasterize_gaussians_backward_ex(
        tt(h["_bg"]), a["means3D"], a["features"], h["radii"], a["colors"], a["scales"], a["rotations"], 1.0,
        a["cov3D"], tt(cam.view), tt(cam.proj), cam.tanfovx, cam.tanfovy, tt(dc.transpose(1, 2, 0)),
        tt(do.reshape(H, W, 1)), tt(dd.reshape(H, W, 1)), tt(native.reshape(H, W, 21)), a["sh"], 3, tt(cam.campos),
        h["geom"], h["num_rendered"], h["binning"], h["image"], True, False, H, W)
    torch.cuda.synchronize()
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dfeatures", "dL_dcov3D", "dL_dsh",
             "dL_dscales", "dL_drotations"]
    got = {k: v.cpu().numpy().reshape(g_ref[k].shape) for k, v in zip(names, out)}
    if exact:
        for k in names:
            np.testing.assert_array_equal(got[k], g_ref[k], err_msg=k)
    else:
        assert_hip_runs_agree("ex layouts atomic", got, g_ref)


def test_empty_and_culled(hip_ext):
    import torch

    scene, cam = synthetic.small_scene(P=500, S=11, seed=1)
    behind = synthetic.Scene(scene.means3D * np.array([1, 1, -1], np.float32), scene.scales, scene.rotations,
                             scene.opacity, scene.sh, scene.features)
    h = hip_forward(hip_ext, behind, cam, S=11)
    assert h["num_rendered"] == 0
    assert int(h["radii"].abs().sum()) == 0
    np.testing.assert_allclose(h["color"].cpu().numpy(), 1.0)
    np.testing.assert_array_equal(h["opacity"].cpu().numpy(), 0.0)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11)
    g = hip_backward(hip_ext, h, dc, do, dd, df)
    for k, v in g.items():
        assert np.all(v == 0), k
    empty = synthetic.Scene(scene.means3D[:0], scene.scales[:0], scene.rotations[:0], scene.opacity[:0],
                            scene.sh[:0], scene.features[:0])
    h0 = hip_forward(hip_ext, empty, cam, S=11)
    assert h0["num_rendered"] == 0 and h0["radii"].numel() == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("size", [(1, 1), (1, 40), (40, 1), (17, 5), (300, 3)])
def test_thin_frames(hip_ext, size):
    """Frames narrower / shorter than a tile (one partial tile row or column: the blends' inside
    tests, the 4-tile-row xyz / normal workgroup and its edge-clamped halo, the padded launch grid):
    forward bit-exact where the default frame is, gradients at the usual bar."""
    W, H = size
    scene, cam = synthetic.small_scene(P=400, S=11, seed=3, width=W, height=H)
    h = hip_forward(hip_ext, scene, cam, S=11)
    o = _oracle_fwd(scene, cam, 11)
    _check_forward(h, o, 11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=W + H)
    gh = hip_backward(hip_ext, h, dc, do, dd, df)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    grad_check(f"thin {W}x{H}", gh, go)


def test_sh_degrees(hip_ext):
    scene, cam = synthetic.small_scene(P=1500, S=3, seed=30, width=64, height=48)
    for deg in range(4):
        h = hip_forward(hip_ext, scene, cam, S=3, degree=deg)
        o = _oracle_fwd(scene, cam, 3, degree=deg)
        _check_forward(h, o, 3)
        dc, do, dd, df = upstream_grads(cam.height, cam.width, 3, seed=deg)
        gh = hip_backward(hip_ext, h, dc, do, dd, df)
        go = oracle.rasterize_backward(o, dc, do, dd, df)
        grad_check(f"sh deg{deg}", gh, go, ["dL_dsh"])


def _keys_vs_oracle(hip_ext, scene, cam, h):
    """Sorted keys (tile << 32 | depth bits) and point list of a HIP forward against the oracle's
    preprocess + duplicateWithKeys + stable sort (rasterizer_impl.cu:343-383); ranges against the
    boundaries of the sorted keys."""
    import ctypes

    import relightable3dgaussian_amd as r

    L = h["num_rendered"]
    st = r._C.rasterizer_state(h["geom"], h["binning"], h["image"], scene.P, cam.height, cam.width, L)
    keys = st[0].cpu().numpy().view(np.uint64)
    lib = oracle.lib()
    P = scene.P
    F = np.float32
    radii = np.zeros(P, np.int32); means2D = np.zeros((P, 2), F); depths = np.zeros(P, F)
    cov3D = np.zeros((P, 6), F); rgb = np.zeros((P, 3), F); cl = np.zeros(P, np.uint8)
    conic = np.zeros((P, 4), F); touched = np.zeros(P, np.uint32)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    sh = np.ascontiguousarray(scene.sh)
    lib.oracle_preprocess(ctypes.c_int(P), ctypes.c_int(3), ctypes.c_int(16), p(scene.means3D), p(scene.scales),
                          ctypes.c_float(1.0), p(scene.rotations), p(scene.opacity.reshape(-1)), p(sh), None, None,
                          p(np.ascontiguousarray(cam.view, F)), p(np.ascontiguousarray(cam.proj, F)),
                          p(np.ascontiguousarray(cam.campos, F)), ctypes.c_int(cam.width), ctypes.c_int(cam.height),
                          ctypes.c_float(cam.tanfovx), ctypes.c_float(cam.tanfovy), p(radii), p(means2D), p(depths),
                          p(cov3D), p(rgb), p(cl), p(conic), p(touched))
    np.testing.assert_array_equal(h["radii"].cpu().numpy(), radii)
    assert int(touched.sum(dtype=np.int64)) == L
    offsets = np.cumsum(touched, dtype=np.uint64).astype(np.uint32)
    okeys = np.zeros(L, np.uint64); ovals = np.zeros(L, np.uint32)
    lib.oracle_duplicate_with_keys(ctypes.c_int(P), p(means2D), p(depths), p(offsets), p(radii),
                                   ctypes.c_int(cam.width), ctypes.c_int(cam.height), p(okeys), p(ovals))
    order = np.lexsort((np.arange(L), okeys))  # stable sort by key
    np.testing.assert_array_equal(keys, okeys[order])
    np.testing.assert_array_equal(st[1].cpu().numpy().view(np.uint32), ovals[order])
    T = ((cam.width + 15) // 16) * ((cam.height + 15) // 16)
    tiles = (okeys[order] >> np.uint64(32)).astype(np.int64)
    lo = np.searchsorted(tiles, np.arange(T), "left")
    hi = np.searchsorted(tiles, np.arange(T), "right")
    rng = np.where((hi > lo)[:, None], np.stack([lo, hi], 1), 0)
    np.testing.assert_array_equal(st[2].cpu().numpy().astype(np.int64), rng)
    return L


def test_m1_keys_full_size(hip_ext):
    """BASELINE.json metric config (1M Gaussians, 1920x1080): keys, sort order and ranges bit-exact
    vs the oracle's preprocess + stable sort; blend invariants checked on the full image."""
    cam = synthetic.m1_camera()
    scene = synthetic.m1_scene(P=1_000_000, S=11, seed=0, cam=cam)
    h = hip_forward(hip_ext, scene, cam, S=11)
    L = _keys_vs_oracle(hip_ext, scene, cam, h)
    assert 4_000_000 < L < 6_500_000
    import torch

    op = h["opacity"].cpu().numpy()[..., 0].reshape(-1)
    fT = h["image"][: cam.height * cam.width * 4].view(torch.float32).cpu().numpy()  # final_T (image state)
    # sum of blend weights + final transmittance == 1 (size-independent invariant)
    assert np.abs(op + fT - 1.0).max() < 2e-5
    assert op.min() >= 0.0 and op.max() <= 1.0


# ------------------------------------------------------------------------------------------------
# render equation
# ------------------------------------------------------------------------------------------------
def _brdf_tensors(inp):
    from tests._helpers import tt

    return [tt(inp[k]) for k in ["base", "rough", "metal", "normals", "viewdirs", "incidents", "env", "visibility"]]



@pytest.mark.parametrize("size", [(3200, 1800), (4200, 2400), (7680, 4320)])
def test_binning_large_frames(hip_ext, size):
    """Binning above 12288 tiles (3200x1800: 22600 tiles, LDS counters beyond 64 KiB per workgroup),
    above kBinMaxTiles (4200x2400: 39450 tiles, the global-atomic fallback) and above 40960 tiles
    (7680x4320: 129600 tiles, tile_ranges_kernel's re-reading PER = 0 path): keys, point list and
    ranges bit-exact vs the oracle."""
    cam = synthetic.m1_camera(*size)
    scene = synthetic.m1_scene(P=150_000, S=3, seed=5, cam=cam)
    h = hip_forward(hip_ext, scene, cam, S=3)
    assert _keys_vs_oracle(hip_ext, scene, cam, h) > 100_000


@rows_reduction()
def test_binning_atomic_path_matches(hip_ext):
    """The global-atomic binning (test_bin_atomic, the fallback above kBinMaxTiles) and the LDS
    binning give bit-identical sorted lists, images and gradients; both match the oracle's keys."""
    cam = synthetic.m1_camera(480, 272)
    scene = synthetic.m1_scene(P=60_000, S=11, seed=9, cam=cam)
    a = hip_forward(hip_ext, scene, cam, S=11)
    _keys_vs_oracle(hip_ext, scene, cam, a)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=2)
    ga = hip_backward(hip_ext, a, dc, do, dd, df)
    with lib_options(test_bin_atomic=1):
        b = hip_forward(hip_ext, scene, cam, S=11)
        gb = hip_backward(hip_ext, b, dc, do, dd, df)
    _keys_vs_oracle(hip_ext, scene, cam, b)
    for k in ["color", "opacity", "depth", "feature", "n_contrib"]:
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)
    for k in ga:
        np.testing.assert_array_equal(ga[k], gb[k], err_msg=k)


@rows_reduction()
@pytest.mark.parametrize("size", [(480, 272), (1920, 1080)])
def test_binning_one_pass_matches(hip_ext, size):
    """The two-pass scatter through 16-tile buckets (default) and the one-pass scatter
    (test_bin_one_pass) give bit-identical sorted lists, ranges, images and gradients; both match the
    oracle's keys. 480x272: 510 tiles, a partial last bucket."""
    cam = synthetic.m1_camera(*size)
    scene = synthetic.m1_scene(P=60_000, S=11, seed=13, cam=cam)
    a = hip_forward(hip_ext, scene, cam, S=11)
    _keys_vs_oracle(hip_ext, scene, cam, a)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=3)
    ga = hip_backward(hip_ext, a, dc, do, dd, df)
    with lib_options(test_bin_one_pass=1):
        b = hip_forward(hip_ext, scene, cam, S=11)
        gb = hip_backward(hip_ext, b, dc, do, dd, df)
    _keys_vs_oracle(hip_ext, scene, cam, b)
    for k in ["color", "opacity", "depth", "feature", "n_contrib"]:
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)
    for k in ga:
        np.testing.assert_array_equal(ga[k], gb[k], err_msg=k)


def test_brdf_complex_matches_oracle_and_golden(hip_ext):
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "brdf_pi5.npz"))
    inp = {k: g[k] for k in ["base", "rough", "metal", "normals", "viewdirs", "incidents", "visibility", "env"]}
    out = hip_ext.render_equation_forward_complex(*_brdf_tensors(inp), 24)
    names = ["pbr", "incident_dirs", "incident_lights", "local_incident_lights", "global_incident_lights",
             "incident_visibility", "diffuse_light", "local_diffuse_light", "accum", "rgb_d", "rgb_s"]
    h = {k: v.cpu().numpy() for k, v in zip(names, out)}
    o = oracle.brdf_forward_complex(inp, 24)
    for k in names:
        assert_brdf(k, h[k], o[k])
    for k in ["pbr", "diffuse_light", "incident_dirs", "incident_lights", "incident_visibility"]:
        assert_close("golden " + k, h[k], g[k], 5e-5, 2e-4)


def test_brdf_training_forward_with_rand(hip_ext):
    inp = synthetic.brdf_inputs(3000, seed=3)
    rnd = np.random.default_rng(9).uniform(0, 1, (3000, 24, 1)).astype(np.float32)
    from tests._helpers import tt

    out = hip_ext.render_equation_forward_with_rand(*_brdf_tensors(inp), 24, True, tt(rnd))
    o = oracle.brdf_forward(inp, 24, True, rnd)
    # random rotation angles up to ~2pi + 24*delta through the shared r3dg_sincosf
    for k, v in zip(["pbr", "incident_dirs", "diffuse_light"], out):
        assert_brdf(k, v.cpu().numpy(), o[k])
    # the reference draws the rotation itself when training: directions must change, stay unit
    pbr, dirs, dl = hip_ext.render_equation_forward(*_brdf_tensors(inp), 24, True, False)
    d = dirs.cpu().numpy()
    assert np.abs(np.linalg.norm(d, axis=-1) - 1).max() < 1e-5


@pytest.mark.parametrize("S", [16, 9])
def test_brdf_backward_matches_oracle(hip_ext, S):
    from tests._helpers import tt

    inp = synthetic.brdf_inputs(4000, seed=5, S=S)
    fw = oracle.brdf_forward(inp, 24)
    rng = np.random.default_rng(6)
    gp = rng.normal(size=(4000, 3)).astype(np.float32)
    gd = rng.normal(size=(4000, 3)).astype(np.float32)
    out = hip_ext.render_equation_backward(*_brdf_tensors(inp), 24, tt(fw["incident_dirs"]), tt(gp), tt(gd), False)
    o = oracle.brdf_backward(inp, fw["incident_dirs"], gp, gd, 24)
    for k, v in zip(["base", "rough", "metal", "normals", "viewdirs", "incidents", "env", "visibility"], out):
        assert_brdf("d_" + k, v.cpu().numpy(), o[k], summed=k == "env")


def test_brdf_backward_golden(hip_ext):
    """Gradient fixture from the reference's autograd (no clamp active): pins the kernel formulas."""
    from tests._helpers import tt

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "brdf_pi5.npz"))
    inp = {k: g["g_" + k] for k in ["base", "rough", "metal", "normals", "viewdirs", "incidents", "visibility", "env"]}
    ones = np.ones((inp["base"].shape[0], 3), np.float32)
    out = hip_ext.render_equation_backward(*_brdf_tensors(inp), 24, tt(g["g_incident_dirs"]), tt(ones), tt(ones),
                                           False)
    names = ["base", "rough", "metal", "normals", "viewdirs", "incidents", "env", "visibility"]
    h = dict(zip(names, (v.cpu().numpy() for v in out)))
    for k in ["base", "rough", "metal", "incidents", "visibility", "env"]:
        ref = g["grad_" + k]
        assert_close("golden d_" + k, h[k], ref, 1e-5 * float(np.abs(ref).max()) + 1e-6, 1e-3)


def test_mark_visible(hip_ext):
    from tests._helpers import tt

    scene, cam = synthetic.small_scene(P=3000, seed=4)
    m = scene.means3D.copy()
    m[::3, 2] *= -1
    v = hip_ext.mark_visible(tt(m), tt(cam.view), tt(cam.proj)).cpu().numpy()
    np.testing.assert_array_equal(v, oracle.mark_visible(m, cam.view))


def test_shader_managers(hip_ext):
    import torch

    from tests._helpers import tt

    scene, cam = synthetic.small_scene(P=3000, seed=4)
    # every splat in the default region of SelectShadersCUDA (y < -0.3, x < -0.6)
    xyz = np.tile(np.array([[-1.0, -1.0, 0.0]], np.float32), (100, 1))
    sh_m, sp_m = hip_ext.PreprocessModel(tt(xyz))
    handles, counts = hip_ext.shader_manager_info(sh_m)
    names = {v: k for k, v in hip_ext.GetShShaderAddressMap().items()}
    assert {names[h]: c for h, c in zip(handles, counts)}["ShDefault"] == 100
    # the reference's position rules: mixed assignment
    xyz2 = np.array([[-1, -1, 0], [0.5, 0.5, 0], [-0.3, 0.0, 0], [0.2, -0.5, 0]], np.float32)
    a, b = hip_ext.PreprocessModel(tt(xyz2))
    sp_names = {v: k for k, v in hip_ext.GetSplatShaderAddressMap().items()}
    hs, cs = hip_ext.shader_manager_info(b)
    got = {sp_names[h]: c for h, c in zip(hs, cs) if c}
    assert got == {"SplatDefault": 1, "Dissolve": 1, "Wireframe": 1, "NaiveOutline": 1}
    # rendering with an all-default manager is the default path; non-default is refused loudly
    from tests._helpers import hip_forward as hf

    base = hf(hip_ext, scene, cam, S=11)
    args = base["_args"]
    out = hip_ext.rasterize_gaussians(tt((1, 1, 1)), 0.0, 0.0, args["means3D"], args["features"], args["colors"],
                                      args["opacity"], args["scales"], args["rotations"], 1.0, args["cov3D"],
                                      tt(cam.view), tt(cam.view_inv), tt(cam.proj), tt(cam.proj_inv), cam.tanfovx,
                                      cam.tanfovy, cam.cx, cam.cy, cam.height, cam.width, args["sh"], 3,
                                      tt(cam.campos), False, True, 0, sh_m, sp_m, [], False)
    np.testing.assert_array_equal(out[2].cpu().numpy(), base["color"].cpu().numpy())
    with pytest.raises(RuntimeError):
        hip_ext.rasterize_gaussians(tt((1, 1, 1)), 0.0, 0.0, args["means3D"], args["features"], args["colors"],
                                    args["opacity"], args["scales"], args["rotations"], 1.0, args["cov3D"],
                                    tt(cam.view), tt(cam.view_inv), tt(cam.proj), tt(cam.proj_inv), cam.tanfovx,
                                    cam.tanfovy, cam.cx, cam.cy, cam.height, cam.width, args["sh"], 3,
                                    tt(cam.campos), False, True, 0, a, b, [], False)
    torch.cuda.synchronize()


def test_autograd_wrapper(hip_ext):
    """Drop-in wrapper: 11-output forward, 11-grad backward, HWC grads routed without transposes."""
    import torch

    from relightable3dgaussian_amd.r3dg_rasterization import GaussianRasterizer, settings_from_camera

    scene, cam = synthetic.small_scene(P=2000, S=11, seed=12, width=64, height=48)
    dev = "cuda"
    st = settings_from_camera(cam, (1.0, 1.0, 1.0))
    rast = GaussianRasterizer(st)
    t = lambda a: torch.tensor(a, device=dev, requires_grad=True)  # noqa: E731
    means3D, opac, feats = t(scene.means3D), t(scene.opacity), t(scene.features)
    shs, scales, rots = t(scene.sh), t(scene.scales), t(scene.rotations)
    means2D = torch.zeros_like(means3D, requires_grad=True)
    out = rast(means3D=means3D, means2D=means2D, opacities=opac, shs=shs, scales=scales, rotations=rots,
               features=feats)
    assert len(out) == 11
    num_rendered, n_contrib, color, opacity, depth, stencil, feature, shader, normal, xyz, radii = out
    H, W = cam.height, cam.width
    dc, do, dd, df = upstream_grads(H, W, 11)
    loss = (color * torch.tensor(dc.transpose(1, 2, 0), device=dev)).sum() + \
        (opacity * torch.tensor(do.reshape(H, W, 1), device=dev)).sum() + \
        (depth * torch.tensor(dd.reshape(H, W, 1), device=dev)).sum()
    groups = [1, 1, 3, 3, 3]
    c = 0
    flat = feature.reshape(-1)
    for n in groups:  # the neilf.py style split of the block layout
        blk = flat[H * W * c:H * W * (c + n)].view(H * W, n)
        loss = loss + (blk * torch.tensor(df[c:c + n].reshape(n, H * W).T.copy(), device=dev)).sum()
        c += n
    loss.backward()
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh,
                                 scales=scene.scales, rotations=scene.rotations)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    got = {"dL_dmeans3D": means3D.grad, "dL_dmeans2D": means2D.grad, "dL_dfeatures": feats.grad, "dL_dsh": shs.grad,
           "dL_dopacity": opac.grad, "dL_dscales": scales.grad, "dL_drotations": rots.grad}
    grad_check("autograd", {k: v.cpu().numpy() for k, v in got.items()}, go, list(got))


@pytest.mark.parametrize("reduce", ["atomic", "rows"])
@pytest.mark.parametrize("S", [0, 11, 21, 32])
def test_backward_reductions_match_oracle(hip_ext, S, reduce):
    """Both second stages of the backward's reduction (the bwd_reduce option): the per-(instance, wave)
    rows added straight into the per-Gaussian sums with f32 atomics, and the deterministic partial
    rows + row_sum_kernel, against the oracle; and against each other."""
    scene, cam = synthetic.small_scene(P=3000, S=max(S, 21), seed=60 + S, width=112, height=80)
    o = _oracle_fwd(scene, cam, S)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, S, seed=3)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    with lib_options(bwd_reduce=int(reduce == "rows")):
        gh = hip_backward(hip_ext, hip_forward(hip_ext, scene, cam, S=S), dc, do, dd, df)
    with lib_options(bwd_reduce=int(reduce != "rows")):
        gx = hip_backward(hip_ext, hip_forward(hip_ext, scene, cam, S=S), dc, do, dd, df)
    grad_check(f"reductions {reduce} S={S}", gh, go)
    for k in go:
        if k in gh:
            assert_close(f"{reduce} vs other {k}", gh[k], gx[k], 1e-6 * max(float(np.abs(gx[k]).max()) if gx[k].size
                                                                           else 0.0, 1e-12), 1e-4)


@pytest.mark.parametrize("S", [11, 21])
def test_backward_mfma_matches_dpp_variant(hip_ext, S):
    """The MFMA reduction (default) and the DPP wave-reduction cross-check of the backward blend
    agree. Each variant runs on a fresh forward: the row flags the backward sets live in the
    forward's binning state, so a stale flag from another call could not hide a missing row."""
    scene, cam = synthetic.small_scene(P=3000, S=21, seed=40 + S, width=96, height=80)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, S)
    gm = hip_backward(hip_ext, hip_forward(hip_ext, scene, cam, S=S), dc, do, dd, df)
    with lib_options(test_bwd_dpp=1):
        gd = hip_backward(hip_ext, hip_forward(hip_ext, scene, cam, S=S), dc, do, dd, df)
    for k in gm:
        assert_close(f"dpp {k}", gm[k], gd[k], 1e-5 * max(float(np.abs(gd[k]).max()) if gd[k].size else 0.0, 1e-12),
                     1e-3)


@pytest.mark.parametrize("reduce", ["rows", "atomic"])
def test_backward_chunked_delivery(hip_ext, reduce):
    """Chunked per-Gaussian phase (r3dg_backward_outputs.n_chunks / chunk_done): the same gradients
    as one chunk (bitwise on the rows reduction, within assert_hip_runs_agree on the default atomic
    flush); the callback sees 256-aligned ranges covering every Gaussian in order, with the output
    tensors (view_parallel.backward_all_reduce overlaps the exchange with it)."""
    if reduce == "rows":
        with rows_reduction():
            _chunked_delivery(hip_ext, exact=True)
    else:
        _chunked_delivery(hip_ext, exact=False)


def _chunked_delivery(hip_ext, exact):
    scene, cam = synthetic.small_scene(P=3000, S=11, seed=77, width=96, height=80)
    h = hip_forward(hip_ext, scene, cam, S=11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11)
    ref = hip_backward(hip_ext, h, dc, do, dd, df)
    a = h["_args"]
    seen = []

    def hook(c, g0, g1, outs):
        seen.append((c, g0, g1, len(outs)))

    args = (tt(h["_bg"]), a["means3D"], a["features"], h["radii"], a["colors"], a["scales"], a["rotations"], 1.0,
            a["cov3D"], tt(cam.view), tt(cam.proj), cam.tanfovx, cam.tanfovy, tt(dc), tt(do), tt(dd), tt(df), a["sh"],
            3, tt(cam.campos), h["geom"], h["num_rendered"], h["binning"], h["image"], True, False, cam.height,
            cam.width, False, False)
    out = hip_ext.rasterize_gaussians_backward_chunked(*args, 5, hook)
    P = scene.P
    assert [s[0] for s in seen] == list(range(len(seen))) and len(seen) > 1
    assert seen[0][1] == 0 and seen[-1][2] == P and all(s[3] == 9 for s in seen)
    assert all(a[2] == b[1] for a, b in zip(seen, seen[1:])) and all(s[1] % 256 == 0 for s in seen)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dfeatures", "dL_dcov3D", "dL_dsh",
             "dL_dscales", "dL_drotations"]
    got = {k: out[i].cpu().numpy().reshape(ref[k].shape) for i, k in enumerate(names)}
    if exact:
        for k in names:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    else:
        assert_hip_runs_agree("chunked atomic", got, ref)


def _chunked_exchange_worker(rank, world, port, q, mode="views"):
    import torch
    import torch.distributed as dist

    import relightable3dgaussian_amd as r3

    r3._C.set_options({"bwd_reduce": 1})  # local and exchanged backward runs are compared bitwise
    from relightable3dgaussian_amd import view_parallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene, cam = synthetic.small_scene(P=2500, S=11, seed=91, width=96, height=80)
    h = hip_forward(r3._C, scene, cam, S=11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11)
    local = hip_backward(r3._C, h, dc, do, dd, df)
    a = h["_args"]
    args = (tt(h["_bg"]), a["means3D"], a["features"], h["radii"], a["colors"], a["scales"], a["rotations"], 1.0,
            a["cov3D"], tt(cam.view), tt(cam.proj), cam.tanfovx, cam.tanfovy, tt(dc), tt(do), tt(dd), tt(df), a["sh"],
            3, tt(cam.campos), h["geom"], h["num_rendered"], h["binning"], h["image"], True, False, cam.height,
            cam.width, False, False)
    out = view_parallel.backward_all_reduce(r3._C, args, n_chunks=4, sh_exchange=mode)
    torch.cuda.synchronize()
    # one collective per chunk for the packed dense rows (+ one for the SH part), + the camera gather
    seq = view_parallel.LAST_COLLECTIVES["sequence"]
    assert len(seq) == (9 if mode == "views" else 8), seq
    assert sum(n for k, n in seq if k == "all_reduce") == 2500 * ((11 + 11) if mode == "views" else (22 + 48))
    res = {name: out[i].cpu().numpy() for name, i in view_parallel.GRAD_FIELDS}
    q.put((rank, res, {"means3D": local["dL_dmeans3D"], "sh": local["dL_dsh"], "opacity": local["dL_dopacity"],
                       "scales": local["dL_dscales"], "rotations": local["dL_drotations"],
                       "features": local["dL_dfeatures"]}))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["views", "allreduce"])
def test_view_parallel_chunked_exchange_two_ranks(hip_ext, mode):
    """bench.py's N > 1 path on one GPU: two gloo ranks render the same view, the chunked
    exchange (overlapped with the gather phase) must return exactly 2x the local gradients --
    also the SH block rebuilt from the all-gathered colour gradients ("views": each view's
    product rounded as the backward rounds it, summed in view order)."""
    import multiprocessing as mp
    import socket

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_chunked_exchange_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, res, local in got:
        for k, v in res.items():
            np.testing.assert_array_equal(v.reshape(local[k].shape), 2 * local[k], err_msg=f"rank {rank} {k}")


def test_sh_rebuild_kernels_match_oracle(hip_ext):
    """r3dg_sh_color_grads + r3dg_sh_grad_from_views (the view-parallel SH exchange) against
    oracle/view_exchange.py and the sum of the C oracle's per-view dL_dsh, three views, chunked
    rows."""
    import torch

    from oracle import view_exchange
    from relightable3dgaussian_amd import view_parallel

    base = synthetic.m1_camera(96, 64)
    scene = synthetic.m1_scene(P=3000, S=11, seed=12, cam=base)
    drgb, cams, per_view_sh = [], [], []
    for r in range(3):
        cam = view_parallel.rank_camera(base, r, 3, step_deg=5.0)
        h = hip_forward(hip_ext, scene, cam, S=11)
        dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=20 + r)
        g = hip_backward(hip_ext, h, dc, do, dd, df)
        o = _oracle_fwd(scene, cam, 11)
        d = hip_ext.sh_color_grads(h["geom"], scene.P, tt(g["dL_dcolors"]), 0, scene.P)
        np.testing.assert_array_equal(d.cpu().numpy(), view_exchange.sh_color_grads(g["dL_dcolors"], o["clamped"]))
        drgb.append(d)
        cams.append(np.asarray(cam.campos, np.float32))
        per_view_sh.append(g["dL_dsh"])
    P = scene.P
    out = torch.full((P, 16, 3), float("nan"), device="cuda")
    d_all = torch.stack(drgb)
    for g0, g1 in [(0, 1024), (1024, 2048), (2048, P)]:
        hip_ext.sh_grad_from_views(tt(scene.means3D), tt(np.stack(cams)), d_all[:, g0:g1].contiguous(), 3, g0, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref = view_exchange.sh_grad_from_views(scene.means3D, np.stack(cams), d_all.cpu().numpy(), 3, 16)
    scale = float(np.abs(ref).max())
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * scale)
    np.testing.assert_allclose(got, sum(per_view_sh), rtol=1e-5, atol=1e-6 * scale)


@lib_options(bwd_reduce=0)
def test_one_term_reduction_fails_bar(hip_ext):
    """The gradient bar can fail: at an M1 crop (480x272 of the M1 camera, the M1 density: 63k
    Gaussians) the default backward (atomic flush, w split into two bf16 terms) meets GRAD_BARS,
    while the one-term reduction (test_bwd_wterms = 1: w truncated to one bf16 term, ~2^-8 relative
    per product) must violate them on the colour / feature gradients. (The wterms switch exists on
    the atomic flush only: the test pins that reduction even when the suite runs under
    R3DG_BWD_REDUCE=rows.)"""
    cam = synthetic.m1_camera(480, 272)
    scene = synthetic.m1_scene(P=63_000, S=11, seed=4, cam=cam)
    o = _oracle_fwd(scene, cam, 11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=8)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    h = hip_forward(hip_ext, scene, cam, S=11)
    _check_forward(h, o, 11)
    grad_check("m1crop", hip_backward(hip_ext, h, dc, do, dd, df), go)
    with lib_options(test_bwd_wterms=1):
        g1 = hip_backward(hip_ext, h, dc, do, dd, df)
    with lib_options(test_bwd_wterms=3):  # the exact split, for the record: the default's
        grad_check("m1crop exact-split", hip_backward(hip_ext, h, dc, do, dd, df), go)  # error above it is the split's
    failed = []
    for k in ["dL_dcolors", "dL_dfeatures"]:
        try:
            grad_check("m1crop one-term", g1, go, [k])
        except AssertionError:
            failed.append(k)
    assert failed == ["dL_dcolors", "dL_dfeatures"], failed


def test_backward_uses_sums_prepared_by_forward(hip_ext):
    """A training forward zeroes the backward's atomic sums inside its blend (RenderFwdArgs::zero_sums,
    no memset launch in the backward). The first backward on that forward uses them; a second one on
    the same forward finds them used and zeroes scratch itself: both agree with each other and with
    the oracle, also on a second forward at the same size."""
    scene, cam = synthetic.small_scene(P=3000, S=11, seed=52, width=112, height=80)
    o = _oracle_fwd(scene, cam, 11)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 11, seed=9)
    go = oracle.rasterize_backward(o, dc, do, dd, df)
    with lib_options(bwd_reduce=0):
        h = hip_forward(hip_ext, scene, cam, S=11)
        g1 = hip_backward(hip_ext, h, dc, do, dd, df)   # the prepared sums
        g2 = hip_backward(hip_ext, h, dc, do, dd, df)   # used: memset path
        h2 = hip_forward(hip_ext, scene, cam, S=11)
        g3 = hip_backward(hip_ext, h2, dc, do, dd, df)
    for g in (g1, g2, g3):
        grad_check("prepared sums", g, go)
    assert_hip_runs_agree("prepared vs memset", g1, g2)
    assert_hip_runs_agree("second forward", g1, g3)
