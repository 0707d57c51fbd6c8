"""BVH visibility tracer: reference bvh/__init__.py, bvh/src/*.cu.

CPU tests pin the oracle (oracle/r3dg_bvh.c): leaf boxes against the reference's own torch code
(tests/golden/bvh.npz), the tree by its structural invariants, the opacity trace against a
brute-force pass over every Gaussian. GPU tests compare the HIP path (`_C.create_bvh`,
`_C.trace_bvh_opacity`, `_C.trace_bvh`, `RayTracer`) with the oracle on the same inputs:
bit-exact for the tree (nodes, boxes, Morton keys) and the trace_bvh lists; the opacity trace
uses __expf like the reference, so visibility is compared at 2e-5 absolute and `contribute`
exactly except on rays whose transmittance sits within 1e-4 of the 0.9 cut.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
F = np.float32


def scene(P, seed=0, spread=1.0, clustered=False, dup=0):
    rng = np.random.default_rng(seed)
    if clustered:  # a few dense clumps: deep, unbalanced Morton trees
        centers = rng.uniform(-spread, spread, (8, 3))
        means = centers[rng.integers(0, 8, P)] + rng.normal(0, 0.01 * spread, (P, 3))
    else:
        means = rng.uniform(-spread, spread, (P, 3))
    if dup:  # identical centres -> identical Morton codes, ties broken by Gaussian index
        means[-dup:] = means[0]
    scales = np.exp(rng.uniform(np.log(0.004), np.log(0.04), (P, 3))) * spread
    rots = rng.normal(size=(P, 4))
    rots /= np.linalg.norm(rots, axis=1, keepdims=True)
    opac = rng.uniform(0.05, 0.95, P)
    opac[rng.random(P) < 0.05] = 0.002  # below 1/255: skipped
    normals = rng.normal(size=(P, 3))
    normals /= np.linalg.norm(normals, axis=1, keepdims=True)
    f = lambda a: np.ascontiguousarray(a, dtype=F)  # noqa: E731
    return dict(means=f(means), scales=f(scales), rots=f(rots), opacity=f(opac), normals=f(normals),
                cov_inv=f(oracle.cov3d(1.0 / f(scales), f(rots))))


def near_cut(t_last, nterms):
    """Rays whose transmittance lies within rounding reach of the 0.9 cut: the GPU (__expf, the
    group's product order) and the oracle (expf, one chain) may legitimately decide them apart.
    The window is the per-factor rounding budget (2e-7, bvh.hip kLogSlack) times the factors
    multiplied, plus 2e-6 -- not a fixed 1e-4."""
    return np.abs(t_last.astype(np.float64) - 0.9) <= 2e-7 * nterms + 2e-6


def rays_from(sc, R, seed=1):
    """The call sites' rays: from Gaussian centres, random directions flipped into the normal's
    hemisphere (neilf.py:329-334, gaussian_model.py:457-460)."""
    rng = np.random.default_rng(seed)
    P = sc["means"].shape[0]
    idx = rng.integers(0, P, R)
    o = sc["means"][idx]
    d = rng.normal(size=(R, 3)).astype(F)
    n = sc["normals"][idx]
    d[(d * n).sum(-1) < 0] *= -1
    return np.ascontiguousarray(o), np.ascontiguousarray(d)


# ---- oracle (CPU) ------------------------------------------------------------------------------

def test_oracle_leaf_boxes_match_reference_torch_code():
    import torch

    g = np.load(os.path.join(HERE, "golden", "bvh.npz"))
    P = g["means3D"].shape[0]
    ours = oracle.bvh_leaf_aabbs(g["means3D"], g["scales"], g["rotations"])
    ref = g["aabbs_init"][P - 1:]
    # torch's CPU sqrt is not correctly rounded on every input (1 ulp); the reference's CUDA
    # torch.sqrt and this build (GPU and oracle) are. Those rows agree to 1 ulp of the box size.
    r = g["rotations"]
    s = r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3]
    cr = torch.sqrt(torch.from_numpy(s)).numpy() == np.sqrt(s)
    assert cr.sum() > P - 20
    assert np.array_equal(ours[cr].view(np.uint32), ref[cr].view(np.uint32))
    np.testing.assert_allclose(ours[~cr], ref[~cr], rtol=0, atol=4e-7)
    # the reference's initial tables: internal rows count 0, leaf rows count 1, boxes +-1e5
    assert (g["nodes_init"][:P - 1, 4] == 0).all() and (g["nodes_init"][P - 1:, 4] == 1).all()
    assert (g["aabbs_init"][:P - 1, :3] == 1e5).all() and (g["aabbs_init"][:P - 1, 3:] == -1e5).all()


def check_tree(nodes, aabbs, keys, P):
    ni = P - 1
    assert nodes.shape == (2 * P - 1, 5) and aabbs.shape == (2 * P - 1, 6) and keys.shape == (P,)
    assert (np.diff(keys.astype(np.uint64)) > 0).all() if P > 1 else True
    assert sorted(nodes[ni:, 3].tolist()) == list(range(P))  # leaves: a permutation of the Gaussians
    assert (keys & np.uint64((1 << 31) - 1)).astype(np.int64).tolist() == nodes[ni:, 3].tolist()
    assert nodes[0, 0] == -1
    if P == 1:
        return
    assert (nodes[ni:, 1:3] == -1).all() and (nodes[ni:, 4] == 1).all() and (nodes[:ni, 3] == -1).all()
    children = nodes[:ni, 1:3].reshape(-1)
    assert sorted(children.tolist()) == list(range(1, 2 * P - 1))  # every node but the root once
    for p in range(ni):
        for c in nodes[p, 1:3]:
            assert nodes[c, 0] == p
        lc, rc = nodes[p, 1], nodes[p, 2]
        assert nodes[p, 4] == nodes[lc, 4] + nodes[rc, 4]
        np.testing.assert_array_equal(aabbs[p, :3], np.minimum(aabbs[lc, :3], aabbs[rc, :3]))
        np.testing.assert_array_equal(aabbs[p, 3:], np.maximum(aabbs[lc, 3:], aabbs[rc, 3:]))


@pytest.mark.parametrize("P,kw", [(1, {}), (2, {}), (3, {}), (37, {}), (2000, {}), (3000, {"clustered": True}),
                                  (500, {"dup": 40})])
def test_oracle_tree_invariants(P, kw):
    sc = scene(P, seed=P, **kw)
    leaf = oracle.bvh_leaf_aabbs(sc["means"], sc["scales"], sc["rots"])
    nodes, aabbs, keys = oracle.bvh_build(leaf)
    check_tree(nodes, aabbs, keys, P)
    np.testing.assert_array_equal(aabbs[P - 1:], leaf[nodes[P - 1:, 3]])


def brute_force_opacity(sc, leaf, o, d):
    """Every Gaussian whose box the ray reaches (exit > 0), in Gaussian order, product in f64."""
    P = leaf.shape[0]
    R = o.shape[0]
    vis = np.ones(R)
    cnt = np.zeros(R, np.int64)
    with np.errstate(divide="ignore", invalid="ignore"):
        for r in range(R):
            t0 = (leaf[:, 0:3] - o[r]) / d[r]
            t1 = (leaf[:, 3:6] - o[r]) / d[r]
            tmin = np.minimum(t0, t1).max(1)
            tmax = np.maximum(t0, t1).min(1)
            hit = (tmax >= tmin) & (tmax > 0) if P > 1 else np.ones(1, bool)
            g = np.nonzero(hit)[0]
            g = g[sc["opacity"][g] >= F(1 / 255)]
            g = g[(sc["normals"][g] * d[r]).sum(-1) <= 0]
            c = sc["cov_inv"][g].astype(np.float64)
            C = np.stack([c[:, [0, 1, 2]], c[:, [1, 3, 4]], c[:, [2, 4, 5]]], 1)
            mu = sc["means"][g] - o[r]
            dd = d[r].astype(np.float64)
            t = np.einsum("gij,gi,j->g", C, mu, dd) / np.einsum("gij,i,j->g", C, dd, dd)
            keep = t >= 0.01
            diff = sc["means"][g][keep] - (o[r] + t[keep, None] * dd)
            power = -0.5 * np.einsum("gi,gij,gj->g", diff, C[keep], diff)
            a = sc["opacity"][g][keep][power <= 0] * np.exp(power[power <= 0])
            T = np.prod(1 - a)
            vis[r], cnt[r] = (T, len(a)) if T >= 0.9 else (0.0, 0)
    return cnt, vis


def test_oracle_opacity_trace_matches_brute_force():
    sc = scene(800, seed=3, spread=0.5)
    leaf = oracle.bvh_leaf_aabbs(sc["means"], sc["scales"], sc["rots"])
    nodes, aabbs, _ = oracle.bvh_build(leaf)
    o, d = rays_from(sc, 300)
    cnt, vis, t_last = oracle.bvh_trace_opacity(nodes, aabbs, o, d, sc["means"], sc["cov_inv"], sc["opacity"],
                                                sc["normals"])
    bc, bv = brute_force_opacity(sc, leaf, o, d)
    ok = np.abs(t_last - 0.9) > 1e-4
    assert ok.sum() > 290 and (bv < 1).sum() > 50 and (bv == 0).sum() > 10  # the scene exercises both cases
    np.testing.assert_array_equal(cnt[ok], bc[ok])
    np.testing.assert_allclose(vis[ok], bv[ok], rtol=0, atol=1e-5)


def test_oracle_trace_lists_sorted_and_counted():
    sc = scene(600, seed=5, spread=0.5)
    leaf = oracle.bvh_leaf_aabbs(sc["means"], sc["scales"], sc["rots"])
    nodes, aabbs, _ = oracle.bvh_build(leaf)
    o, d = rays_from(sc, 200, seed=9)
    cnt, point, pos, rid = oracle.bvh_trace(nodes, aabbs, o, d, sc["means"])
    assert len(point) == cnt.sum() > 0
    assert (np.diff(rid) >= 0).all() and np.array_equal(np.bincount(rid, minlength=200), cnt)
    assert ((point >= -1) & (point < 600)).all() and (point >= 0).sum() > 0
    for r in range(200):  # within a ray, accepted points ascend in t; rejected (t = 1e6) come last
        sel = rid == r
        p = point[sel]
        t = np.where(p >= 0, ((sc["means"][np.maximum(p, 0)] - o[r]) * d[r]).sum(-1), 1e6)
        assert (np.diff(t) >= -1e-6).all()


# ---- HIP path (GPU) -----------------------------------------------------------------------------

def tt(a, dtype=None):
    import torch

    return torch.as_tensor(np.ascontiguousarray(a), device="cuda", dtype=dtype)


def hip_build(_C, sc):
    import torch

    P = sc["means"].shape[0]
    nodes = torch.full((2 * P - 1, 5), -1, dtype=torch.int32, device="cuda")
    nodes[:P - 1, 4] = 0
    nodes[P - 1:, 4] = 1
    aabbs = torch.zeros((2 * P - 1, 6), device="cuda")
    aabbs[:, :3] = 100000
    aabbs[:, 3:] = -100000
    leaf = _C.bvh_leaf_aabbs(tt(sc["means"]), tt(sc["scales"]), tt(sc["rots"]))
    aabbs[P - 1:] = leaf
    n, b, m = _C.create_bvh(tt(sc["means"]), tt(sc["scales"]), tt(sc["rots"]), nodes, aabbs)
    torch.cuda.synchronize()
    return leaf.cpu().numpy(), n, b, m


@pytest.mark.gpu
@pytest.mark.parametrize("P,kw", [(1, {}), (2, {}), (3, {}), (37, {}), (5000, {}), (20000, {"clustered": True}),
                                  (3000, {"dup": 200}), (300000, {})])
def test_gpu_build_bit_exact(hip_ext, P, kw):
    sc = scene(P, seed=P + 11, **kw)
    leaf, n, b, m = hip_build(hip_ext, sc)
    ref_leaf = oracle.bvh_leaf_aabbs(sc["means"], sc["scales"], sc["rots"])
    assert np.array_equal(leaf.view(np.uint32), ref_leaf.view(np.uint32))
    rn, rb, rk = oracle.bvh_build(ref_leaf)
    assert np.array_equal(m.cpu().numpy().view(np.uint64), rk)
    assert np.array_equal(n.cpu().numpy(), rn)
    assert np.array_equal(b.cpu().numpy().view(np.uint32), rb.view(np.uint32))
    if P <= 5000:
        check_tree(n.cpu().numpy(), b.cpu().numpy(), m.cpu().numpy().view(np.uint64), P)


def compare_opacity(hip_ext, sc, nodes, aabbs, o, d, sel=None, min_ok=0.999):
    import torch

    c, v = hip_ext.trace_bvh_opacity(nodes, aabbs, tt(o), tt(d), tt(sc["means"]), tt(sc["cov_inv"]),
                                     tt(sc["opacity"]), tt(sc["normals"]))
    torch.cuda.synchronize()
    c, v = c.cpu().numpy(), v.cpu().numpy()
    if sel is not None:
        c, v, o, d = c[sel], v[sel], o[sel], d[sel]
    rc, rv, t_last, nt = oracle.bvh_trace_opacity(nodes.cpu().numpy(), aabbs.cpu().numpy(), o, d, sc["means"],
                                                  sc["cov_inv"], sc["opacity"], sc["normals"], with_terms=True)
    ok = ~near_cut(t_last, nt)
    assert ok.mean() > min_ok
    np.testing.assert_array_equal(c[ok], rc[ok])
    np.testing.assert_allclose(v[ok], rv[ok], rtol=0, atol=2e-5)
    return rc, rv


@pytest.mark.gpu
@pytest.mark.parametrize("P,R", [(1, 50), (2, 50), (3000, 4000), (50000, 20000)])
def test_gpu_trace_opacity_matches_oracle(hip_ext, P, R):
    sc = scene(P, seed=P + 3, spread=0.5)
    _, n, b, _ = hip_build(hip_ext, sc)
    o, d = rays_from(sc, R, seed=P)
    rc, rv = compare_opacity(hip_ext, sc, n, b, o, d)
    if P > 100:
        assert (rv == 0).sum() > 0 and ((rv > 0) & (rv < 1)).sum() > 0


@pytest.mark.gpu
def test_gpu_trace_opacity_output_shapes(hip_ext):
    sc = scene(500, seed=2, spread=0.5)
    _, n, b, _ = hip_build(hip_ext, sc)
    o, d = rays_from(sc, 24)
    c, v = hip_ext.trace_bvh_opacity(n, b, tt(o.reshape(4, 6, 3)), tt(d.reshape(4, 6, 3)), tt(sc["means"]),
                                     tt(sc["cov_inv"]), tt(sc["opacity"][:, None]), tt(sc["normals"]))
    assert tuple(c.shape) == (4, 6) and tuple(v.shape) == (4, 6)
    import torch

    assert c.dtype == torch.int32 and v.dtype == torch.float32
    c0, v0 = hip_ext.trace_bvh_opacity(n, b, tt(o), tt(d), tt(sc["means"]), tt(sc["cov_inv"]), tt(sc["opacity"]),
                                       tt(sc["normals"]))
    assert torch.equal(c.reshape(-1), c0) and torch.equal(v.reshape(-1), v0)


@pytest.mark.gpu
@pytest.mark.parametrize("P,R", [(2, 40), (4, 40), (2000, 3000), (40000, 5000)])
def test_gpu_trace_lists_bit_exact(hip_ext, P, R):
    sc = scene(P, seed=P + 5, spread=0.5)
    _, n, b, _ = hip_build(hip_ext, sc)
    o, d = rays_from(sc, R, seed=P + 1)
    c, point, pos, rid = hip_ext.trace_bvh(n, b, tt(o), tt(d), tt(sc["means"]), tt(sc["cov_inv"]),
                                           tt(sc["opacity"]))
    rc, rp, rpos, rrid = oracle.bvh_trace(n.cpu().numpy(), b.cpu().numpy(), o, d, sc["means"])
    assert tuple(c.shape) == (R, 1)
    assert np.array_equal(c.cpu().numpy()[:, 0], rc)
    assert tuple(point.shape) == (len(rp), 1) and tuple(pos.shape) == (len(rp), 3)
    assert np.array_equal(point.cpu().numpy()[:, 0], rp)
    assert np.array_equal(rid.cpu().numpy()[:, 0], rrid)
    assert np.array_equal(pos.cpu().numpy().view(np.uint32), rpos.view(np.uint32))


@pytest.mark.gpu
def test_gpu_trace_lists_empty(hip_ext):
    sc = scene(300, seed=1, spread=0.5)
    _, n, b, _ = hip_build(hip_ext, sc)
    o = np.full((8, 3), 50.0, F)  # far outside, pointing away
    d = np.tile(np.array([[1.0, 1.0, 1.0]], F), (8, 1))
    c, point, pos, rid = hip_ext.trace_bvh(n, b, tt(o), tt(d), tt(sc["means"]), tt(sc["cov_inv"]), tt(sc["opacity"]))
    assert int(c.sum()) == 0 and tuple(point.shape) == (0, 1) and tuple(pos.shape) == (0, 3)
    assert tuple(rid.shape) == (0, 3)  # the reference's float [0, 3] (bvh.cu:51)


@pytest.mark.gpu
def test_gpu_trace_near_cut_many_faint_hits(hip_ext):
    """Rays built to end near T = 0.9 after ~300 faint hits each (alpha ~ 3e-4): the group's
    early cut (bvh.hip kLogCut / kLogSlack) must never occlude a ray the reference keeps, nor keep
    one it occludes, outside the per-factor rounding window."""
    N, sigma = 300, 0.05
    z = np.linspace(1.0, 4.0, N)
    means = np.stack([np.zeros(N), np.zeros(N), z], 1)
    rots = np.tile(np.array([[1.0, 0.0, 0.0, 0.0]]), (N, 1))
    scales = np.full((N, 3), sigma)
    f = lambda a: np.ascontiguousarray(a, dtype=F)  # noqa: E731
    sc = dict(means=f(means), scales=f(scales), rots=f(rots), opacity=f(np.full(N, 0.005)),
              normals=f(np.tile(np.array([[0.0, 0.0, -1.0]]), (N, 1))),
              cov_inv=f(oracle.cov3d(1.0 / f(scales), f(rots))))
    _, n, b, _ = hip_build(hip_ext, sc)
    R = 8192
    x = np.linspace(0.10, 0.13, R)
    o = f(np.stack([x, np.zeros(R), np.zeros(R)], 1))
    d = f(np.tile(np.array([[0.0, 0.0, 1.0]]), (R, 1)))
    rc, rv, t_last, nt = oracle.bvh_trace_opacity(n.cpu().numpy(), b.cpu().numpy(), o, d, sc["means"], sc["cov_inv"],
                                                  sc["opacity"], sc["normals"], with_terms=True)
    assert nt.max() >= 250 and (rc == 0).any() and (rc > 0).any()
    assert (np.abs(t_last - 0.9) < 1e-4).sum() >= 10  # the scene exercises the cut zone
    compare_opacity(hip_ext, sc, n, b, o, d, min_ok=0.9)  # ~6 % of these rays sit inside the window


@pytest.mark.gpu
def test_gpu_raytracer_call_site(hip_ext):
    """neilf.py:323-348 / gaussian_model.py:446-465 through the drop-in `bvh` module."""
    import torch

    import relightable3dgaussian_amd as r

    r.install_alias()
    from bvh import RayTracer

    sc = scene(20000, seed=21, spread=0.6)
    means, scales, rots = tt(sc["means"]), tt(sc["scales"]), tt(sc["rots"])
    rt = RayTracer(means, scales, rots)
    o, d = rays_from(sc, 10000, seed=4)
    res = rt.trace_visibility(tt(o), tt(d), means, tt(sc["cov_inv"]), tt(sc["opacity"][:, None]),
                              tt(sc["normals"]))
    assert tuple(res["visibility"].shape) == (10000, 1) and tuple(res["contribute"].shape) == (10000, 1)
    leaf = oracle.bvh_leaf_aabbs(sc["means"], sc["scales"], sc["rots"])
    rn, rb, rk = oracle.bvh_build(leaf)
    assert np.array_equal(rt.tree.cpu().numpy(), rn) and np.array_equal(rt.morton.cpu().numpy().view(np.uint64), rk)
    rc, rv, t_last, nt = oracle.bvh_trace_opacity(rn, rb, o, d, sc["means"], sc["cov_inv"], sc["opacity"],
                                                  sc["normals"], with_terms=True)
    ok = ~near_cut(t_last, nt)
    np.testing.assert_array_equal(res["contribute"].cpu().numpy()[ok, 0], rc[ok])
    np.testing.assert_allclose(res["visibility"].cpu().numpy()[ok, 0], rv[ok], rtol=0, atol=2e-5)
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_full_size_build_and_trace(hip_ext):
    """1M Gaussians, 1M rays (finetune_visibility's rays_o = every centre): the whole tree
    bit-exact against the oracle, a 4k-ray sample of the trace against the oracle."""
    sc = scene(1_000_000, seed=8, spread=1.0)
    _, n, b, m = hip_build(hip_ext, sc)
    rn, rb, rk = oracle.bvh_build(oracle.bvh_leaf_aabbs(sc["means"], sc["scales"], sc["rots"]))
    assert np.array_equal(m.cpu().numpy().view(np.uint64), rk)
    assert np.array_equal(n.cpu().numpy(), rn)
    assert np.array_equal(b.cpu().numpy().view(np.uint32), rb.view(np.uint32))
    o, d = rays_from(sc, 1_000_000, seed=2)
    sel = np.random.default_rng(0).choice(1_000_000, 4000, replace=False)
    compare_opacity(hip_ext, sc, n, b, o, d, sel=sel)


def test_create_bvh_refuses_cpu_tensors():
    import torch

    import relightable3dgaussian_amd as r

    with pytest.raises(RuntimeError):
        r._C.create_bvh(torch.zeros(2, 3), torch.zeros(2, 3), torch.zeros(2, 4),
                        torch.zeros(3, 5, dtype=torch.int32), torch.zeros(3, 6))
    with pytest.raises(RuntimeError):
        r._C.bvh_leaf_aabbs(torch.zeros(2, 3), torch.zeros(2, 3), torch.zeros(2, 4))


@pytest.mark.gpu
@pytest.mark.parametrize("lanes,split", [(1, 0), (2, 0), (8, 0), (64, 0), (4, 1), (32, 1)])
def test_gpu_trace_opacity_lane_variants(hip_ext, lanes, split):
    """Every lanes-per-ray setting of both group kernels (shared stack / subtree split) and the
    one-lane reference-order kernel agree with the oracle (r3dg_options test_bvh_lanes / _split)."""
    from tests._helpers import lib_options

    sc = scene(6000, seed=lanes + 10 * split, spread=0.5)
    _, n, b, _ = hip_build(hip_ext, sc)
    o, d = rays_from(sc, 3000, seed=lanes)
    with lib_options(test_bvh_lanes=lanes, test_bvh_split=split):
        compare_opacity(hip_ext, sc, n, b, o, d)
