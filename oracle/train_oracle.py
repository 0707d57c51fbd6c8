"""CPU oracle of the training step on the device -- TEST INFRASTRUCTURE ONLY.

numpy float32 restatement of the reference's training-side per-Gaussian logic that
relightable3dgaussian_amd/csrc/optim.hip replaces. Models are dicts
group name -> [P, width] float32 arrays (the reference's parameters flattened per Gaussian, in
the Adam group order of scene/gaussian_model.py:586-612).

Pinned by tests/golden/train.npz: the reference's own GaussianModel run on CPU
(tests/golden/make_golden_train.py) -- Adam steps, densification statistics,
densify_and_prune with stored noise, reset_opacity.
"""
from __future__ import annotations

import numpy as np

F = np.float32

# scene/gaussian_model.py:586-612 (use_pbr): group name, floats per Gaussian
GROUPS = [("xyz", 3), ("normal", 3), ("rotation", 4), ("scaling", 3), ("opacity", 1), ("f_dc", 3),
          ("f_rest", 45), ("base_color", 3), ("roughness", 1), ("metallic", 1), ("incidents_dc", 3),
          ("incidents_rest", 45), ("visibility_dc", 1), ("visibility_rest", 15)]


def expon_lr(step, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:30-66 get_expon_lr_func (host-side scalar)."""
    if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
        return 0.0
    if lr_delay_steps > 0:
        delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
    else:
        delay_rate = 1.0
    t = np.clip(step / max_steps, 0, 1)
    return float(delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t))


def adam_step(p, g, m, v, lr, step, beta1=0.9, beta2=0.999, eps=1e-15):
    """torch.optim.Adam single-tensor step as the reference calls it (gaussian_model.py:615-617,
    torch/optim/adam.py _single_tensor_adam): returns new (p, m, v). lr is a scalar or per-element."""
    p, g, m, v = (np.asarray(x, F) for x in (p, g, m, v))
    m = (m + F(1 - beta1) * (g - m)).astype(F)                       # exp_avg.lerp_(grad, 1 - beta1)
    v = (v * F(beta2) + F(1 - beta2) * g * g).astype(F)               # mul_(beta2).addcmul_(g, g, 1 - b2)
    bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
    step_size = (np.asarray(lr, np.float64) / bc1).astype(F)
    denom = (np.sqrt(v) / F(bc2 ** 0.5) + F(eps)).astype(F)
    return (p - step_size * (m / denom)).astype(F), m, v


def densification_stats(d2, ngrad, radii, xyz_accum, normal_accum, denom, max_radii):
    """train.py:172-176 + add_densification_stats (gaussian_model.py:1055-1062), in place."""
    vis = radii > 0
    max_radii[vis] = np.maximum(max_radii[vis], radii[vis].astype(F))
    xyz_accum[vis] += np.linalg.norm(d2[vis, :2].astype(F), axis=-1).astype(F)
    if ngrad is not None:
        n = ngrad[vis].astype(F)
        u = n / np.maximum(np.linalg.norm(n, axis=-1, keepdims=True), F(1e-3))  # normalize(eps=1e-3)
        normal_accum[vis] += np.linalg.norm(u, axis=-1).astype(F)
    denom[vis] += F(1)


def _sigmoid(x):
    return (F(1) / (F(1) + np.exp(-x.astype(F)))).astype(F)


def build_rotation(q):
    """utils/general_utils.py:82-103."""
    q = q / np.sqrt((q * q).sum(-1, keepdims=True))
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.zeros((q.shape[0], 3, 3), F)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z); R[:, 0, 1] = 2 * (x * y - r * z); R[:, 0, 2] = 2 * (x * z + r * y)
    R[:, 1, 0] = 2 * (x * y + r * z); R[:, 1, 1] = 1 - 2 * (x * x + z * z); R[:, 1, 2] = 2 * (y * z - r * x)
    R[:, 2, 0] = 2 * (x * z - r * y); R[:, 2, 1] = 2 * (y * z + r * x); R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def densify_and_prune(model, m, v, xyz_accum, normal_accum, denom, max_radii, max_grad, min_opacity, extent,
                      max_screen_size, max_grad_normal, percent_dense, noise, N=2, prune_only=False):
    """densify_and_prune (gaussian_model.py:1025-1043) = densify_and_clone (:982-1023), then
    densify_and_split (:926-980), then the opacity / size prune; or `prune` (:1045-1053) when
    prune_only. model / m / v: dicts name -> [P, w]; returns new (model, m, v)."""
    names = list(model)
    P = model["xyz"].shape[0]
    scale = np.exp(model["scaling"]).astype(F)
    smax = scale.max(1)
    if prune_only:
        clone = split = np.zeros(P, bool)
        mr = max_radii
    else:
        with np.errstate(invalid="ignore", divide="ignore"):
            g = (xyz_accum / denom).astype(F)
            gn = (normal_accum / denom).astype(F)
        g[np.isnan(g)] = 0
        gn[np.isnan(gn)] = 0
        sel = (np.abs(g) >= F(max_grad)) | (np.abs(gn) >= F(max_grad_normal))
        clone = sel & (smax <= F(percent_dense * extent))
        split = sel & (smax > F(percent_dense * extent))
        mr = np.zeros(P, F)  # densification_postfix zeroed max_radii2D before the prune test

    def pruned(op, sm, radius):
        p = _sigmoid(op) < F(min_opacity)
        if max_screen_size:
            p = p | (radius > F(max_screen_size)) | (sm > F(0.1 * extent))
        return p

    op = model["opacity"][:, 0]
    keep_o = ~split & ~pruned(op, smax, mr)
    keep_c = clone & ~pruned(op, smax, mr)
    sidx = np.nonzero(split)[0]
    ns = len(sidx)
    child_scale_raw = np.log(scale[sidx] / F(0.8 * N)).astype(F)
    child_smax = np.exp(child_scale_raw).max(1) if ns else np.zeros(0, F)
    keep_s = ~pruned(op[sidx], child_smax, np.zeros(ns, F))
    # children: xyz = R (std * z) + xyz over the .repeat(N, 1) stack (:940-944)
    z = np.asarray(noise, F)[:3 * N * ns].reshape(N * ns, 3)
    std = np.tile(scale[sidx], (N, 1))
    smp = (F(0) + std * z).astype(F)
    R = np.tile(build_rotation(model["rotation"][sidx]), (N, 1, 1))
    cxyz = (np.einsum("nij,nj->ni", R, smp) + np.tile(model["xyz"][sidx], (N, 1))).astype(F)
    ck = np.tile(keep_s, N)
    out, om, ov = {}, {}, {}
    for k in names:
        a = model[k]
        child = np.tile(a[sidx], (N, 1))
        if k == "xyz":
            child = cxyz
        elif k == "scaling":
            child = np.tile(child_scale_raw, (N, 1))
        out[k] = np.concatenate([a[keep_o], a[keep_c], child[ck]]).astype(F)
        zc = np.zeros((keep_c.sum() + ck.sum(), a.shape[1]), F)
        om[k] = np.concatenate([m[k][keep_o], zc]).astype(F)
        ov[k] = np.concatenate([v[k][keep_o], zc]).astype(F)
    return out, om, ov


def reset_opacity(model, m, v):
    """gaussian_model.py:688-691 (+ replace_tensor_to_optimizer zeroing the opacity state)."""
    y = np.minimum(_sigmoid(model["opacity"]), F(0.01))
    model["opacity"] = np.log(y / (F(1) - y)).astype(F)
    m["opacity"] = np.zeros_like(m["opacity"])
    v["opacity"] = np.zeros_like(v["opacity"])
