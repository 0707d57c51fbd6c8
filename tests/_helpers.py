"""Shared helpers: run the HIP path through `_C` exactly as the reference call sites do."""
from __future__ import annotations

import numpy as np


def tt(a, device="cuda"):
    import torch

    if a is None:
        return torch.empty(0, device=device)
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=device)


def hip_forward(_C, scene, cam, S=None, degree=3, bg=(1.0, 1.0, 1.0), use_sh=True, use_cov=False, colors=None,
                scale_modifier=1.0, pseudo_normal=True, features=None, time=0.0, texture_manager=None,
                sh_manager=None, splat_manager=None, post_passes=None, prefiltered=False):
    """Call _C.rasterize_gaussians with the argument order of rasterize_points.cu:39-71."""
    import torch

    feats = scene.features if features is None else features
    if S is not None:
        feats = feats[:, :S]
    cov = None
    if use_cov:
        import oracle

        cov = oracle.cov3d(scene.scales, scene.rotations, scale_modifier)
    args = dict(
        means3D=tt(scene.means3D), features=tt(np.ascontiguousarray(feats)),
        colors=tt(colors) if colors is not None else tt(None), opacity=tt(scene.opacity),
        scales=tt(None) if use_cov else tt(scene.scales), rotations=tt(None) if use_cov else tt(scene.rotations),
        cov3D=tt(cov) if use_cov else tt(None), sh=tt(scene.sh) if (use_sh and colors is None) else tt(None))
    out = _C.rasterize_gaussians(
        tt(bg), time, 0.0, args["means3D"], args["features"], args["colors"], args["opacity"], args["scales"],
        args["rotations"], scale_modifier, args["cov3D"], tt(cam.view), tt(cam.view_inv), tt(cam.proj),
        tt(cam.proj_inv), cam.tanfovx, cam.tanfovy, cam.cx, cam.cy, cam.height, cam.width, args["sh"], degree,
        tt(cam.campos), prefiltered, pseudo_normal, texture_manager, sh_manager, splat_manager, post_passes,
        False)
    names = ["num_rendered", "n_contrib", "color", "opacity", "depth", "stencil", "feature", "shader_color", "normal",
             "surface_xyz", "radii", "geom", "binning", "image"]
    res = dict(zip(names, out))
    res["_args"] = args
    res["_cam"] = cam
    res["_degree"] = degree
    res["_bg"] = bg
    res["_scale_modifier"] = scale_modifier
    torch.cuda.synchronize()
    return res


def hip_backward(_C, fwd, dcolor_chw, dopac, ddepth, dfeat_planar, backward_geometry=True):
    """_C.rasterize_gaussians_backward with the reference's CHW / planar grad contract."""
    a = fwd["_args"]
    cam = fwd["_cam"]
    out = _C.rasterize_gaussians_backward(
        tt(fwd["_bg"]), a["means3D"], a["features"], fwd["radii"], a["colors"], a["scales"], a["rotations"],
        fwd["_scale_modifier"], a["cov3D"], tt(cam.view), tt(cam.proj), cam.tanfovx, cam.tanfovy, tt(dcolor_chw),
        tt(dopac), tt(ddepth), tt(dfeat_planar), a["sh"], fwd["_degree"], tt(cam.campos), fwd["geom"],
        fwd["num_rendered"], fwd["binning"], fwd["image"], backward_geometry, False)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dfeatures", "dL_dcov3D", "dL_dsh",
             "dL_dscales", "dL_drotations"]
    return {k: v.detach().cpu().numpy() for k, v in zip(names, out)}


def upstream_grads(H, W, S, seed=1, scale=1e-3):
    rng = np.random.default_rng(seed)
    f = lambda *s: (rng.normal(size=s) * scale).astype(np.float32)  # noqa: E731
    return f(3, H, W), f(H * W), f(H * W), f(S, H, W)


def close(a, b, atol, rtol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    return float(err.max()) if err.size else 0.0


def assert_close(name, a, b, atol, rtol=0.0):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, f"{name}: shape {a.shape} vs {b.shape}"
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    bad = d > (atol + rtol * np.abs(b.astype(np.float64)))
    assert not bad.any(), (f"{name}: {int(bad.sum())}/{bad.size} elements off, max abs diff {d.max():.3e} "
                           f"(atol {atol}, rtol {rtol}) at {np.unravel_index(np.argmax(d), d.shape)}")


def assert_brdf(name, got, ref, summed=False):
    """The render equation's outputs against the oracle at north_star's bar: 1e-4 abs, no relative
    slack. brdf.hip and the oracle evaluate the same IEEE operation sequence (shared sin / cos /
    exp statements, contraction off), so every per-Gaussian output is expected bit-identical; the
    count of differing elements is printed. `summed`: dL_ddirect_shs, a sum over every (Gaussian,
    sample) whose order differs (block tree vs the oracle's exact sum): 1e-4 relative to its scale
    (max |ref|)."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    print(f"brdf {name}: {int((got != ref).sum())}/{got.size} differ, max abs diff {d.max() if d.size else 0:.3e}")
    if summed:
        assert_close(name, got, ref, 1e-4 * max(float(np.abs(ref).max()), 1e-12), 1e-4)
    else:
        assert_close(name, got, ref, 1e-4, 0.0)


# ------------------------------------------------------------------------------------------------
# raster-gradient parity (HIP backward vs the oracle)
# ------------------------------------------------------------------------------------------------
def grad_stats(got, ref):
    """(max |got - ref| / max |ref|, the largest elementwise relative error over the elements with
    |ref| > 1e-3 max |ref|): the two numbers a gradient bar is set from."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    if ref.size == 0:
        return 0.0, 0.0
    d = np.abs(got - ref)
    m = float(np.abs(ref).max())
    if m == 0.0:
        return float(d.max()), 0.0
    big = np.abs(ref) > 1e-3 * m
    rel = float((d[big] / np.abs(ref[big])).max()) if big.any() else 0.0
    return float(d.max()) / m, rel


def check_grad(tag, name, got, ref, rel, frac):
    """Assert |got - ref| <= rel |ref| + frac max|ref| elementwise, after printing grad_stats (and
    appending them to $R3DG_GRAD_REPORT as a JSON line, the measurement DESIGN.md §5 records)."""
    import json
    import os

    f, r = grad_stats(got, ref)
    print(f"grad {tag} {name}: max|d|/max|ref| {f:.2e}, max rel (|ref| > 1e-3 max) {r:.2e}")
    path = os.environ.get("R3DG_GRAD_REPORT")
    if path:
        # the smallest frac that passes together with each rel (the bar's trade-off curve)
        g64 = np.asarray(got, np.float64)
        r64 = np.asarray(ref, np.float64)
        m64 = float(np.abs(r64).max()) if r64.size else 0.0
        need = {}
        if m64 > 0:
            d64 = np.abs(g64 - r64)
            for rr in (0.0, 1e-5, 3e-5, 1e-4, 3e-4, 1e-3, 2e-3):
                need[str(rr)] = float(max((d64 - rr * np.abs(r64)).max(), 0.0)) / m64
        with open(path, "a") as fh:
            fh.write(json.dumps({"test": tag, "grad": name, "frac": f, "rel": r, "bar_rel": rel, "bar_frac": frac,
                                 "need_frac": need,
                                 "reduce": "rows" if current_option("bwd_reduce") == 1 else "atomic",
                                 "wterms": current_option("test_bwd_wterms") or 2}) + "\n")
    m = float(np.abs(np.asarray(ref)).max()) if np.asarray(ref).size else 0.0
    assert_close(f"{tag} {name}", got, ref, frac * max(m, 1e-12), rel)


def assert_brdf_refops(name, got, ref, grad=False, summed=False, sensitivity=None):
    """The render equation against the oracle run with the REFERENCE's operation sequence
    (oracle.brdf_reference_ops: libm sinf / cosf / expf / powf, divisions as written) instead of
    the shared statements brdf.hip restates bit for bit: the distance from this build's arithmetic
    to the reference's. Round 3's bars (before the shared statements): outputs 2e-4 abs + 1e-3 rel,
    gradients 2e-5 max|ref| + 1e-3 rel (the summed environment gradient 5e-4 max|ref|).
    `sensitivity(gaussians) -> {gaussian: spread}`: for the few Gaussians outside the bar, the spread
    of the reference-ops oracle itself when its sample directions move by one ulp; such an element
    passes within 4x that spread (ill-conditioned: the sharp lobe at the roughness floor amplifies an
    ulp ~500x and d_rough cancels large terms). At most 1e-4 of the Gaussians may need it."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    m = float(np.abs(ref).max()) if ref.size else 0.0
    atol = ((5e-4 if summed else 2e-5) * max(m, 1e-9)) if grad else 2e-4
    bar = atol + 1e-3 * np.abs(ref.astype(np.float64))
    bad = d > bar
    print(f"brdf vs reference ops {name}: max abs diff {d.max() if d.size else 0:.3e} (max|ref| {m:.3e}), "
          f"{int(bad.sum())} outside round 3's bar")
    if bad.any() and sensitivity is not None and not summed:
        gs = sorted(set(int(i) for i in np.argwhere(bad)[:, 0]))
        assert len(gs) <= max(1, int(1e-4 * ref.shape[0])), (name, len(gs))
        spread = sensitivity(gs)
        for g in gs:
            dg = d[g].max()
            print(f"  {name} Gaussian {g}: diff {dg:.3e}, oracle ulp spread {spread[g]:.3e}")
            assert dg <= 4.0 * spread[g] + bar[g].max(), (name, g, dg, spread[g])
        return
    assert_close(name, got, ref, atol, 1e-3)


import contextlib  # noqa: E402


class lib_options(contextlib.ContextDecorator):
    """Context manager / decorator: library options (r3dg_set_options, include/r3dg_hip.h) for the
    duration, e.g. lib_options(test_no_cull=1); the previous options are restored on exit. The
    library reads no environment variable on a launch: tests switch variants through this API."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        import relightable3dgaussian_amd as r

        self.prev = r._C.set_options(self.kw)
        return self

    def __exit__(self, *exc):
        import relightable3dgaussian_amd as r

        r._C.set_options(self.prev)
        return False


def current_option(name):
    import relightable3dgaussian_amd as r

    return r._C.get_options()[name]


class rows_reduction(lib_options):
    """Context manager / decorator: the backward's deterministic reduction (bwd_reduce = rows: partial rows
    summed in a fixed order) for tests that compare two HIP backward runs bit for bit; the default
    atomic flush is order-dependent in the last bits, as the reference's atomics are."""

    def __init__(self):
        super().__init__(bwd_reduce=1)
