"""PyTorch-CPU restatement of the reference's pure-Python render equation -- TEST / BASELINE
INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline leg). Never imported by the product.

Follows gaussian_renderer/neilf.py:426-519 (sample_incident_rays, rendering_equation_python),
utils/graphics_utils.py:9-37 (fibonacci_sphere_sampling), utils/sh_utils.py:36-66
(rotation_between_z) and :131-170 (eval_sh_coef). It is the reference's CPU path for SURVEY.md
§8d config C1 and the north_star's CPU baseline; the reference Python itself does not travel to
the GPU box. Pinned by tests/golden/brdf.npz (outputs of the reference's own function, np.pi) in
tests/test_oracle.py. `pi` defaults to np.pi like the Python path (the CUDA kernels use 3.14159f).
"""
from __future__ import annotations

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def sh_basis(deg: int, d: torch.Tensor) -> torch.Tensor:
    """Real SH basis up to degree `deg` (<= 3) at unit directions d [..., 3] -> [..., (deg+1)^2]."""
    x, y, z = d[..., 0], d[..., 1], d[..., 2]
    cols = [torch.full_like(x, SH_C0)]
    if deg > 0:
        cols += [-SH_C1 * y, SH_C1 * z, -SH_C1 * x]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        cols += [SH_C2[0] * xy, SH_C2[1] * yz, SH_C2[2] * (2.0 * zz - xx - yy), SH_C2[3] * xz, SH_C2[4] * (xx - yy)]
    if deg > 2:
        cols += [SH_C3[0] * y * (3 * xx - yy), SH_C3[1] * xy * z, SH_C3[2] * y * (4 * zz - xx - yy),
                 SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy), SH_C3[4] * x * (4 * zz - xx - yy),
                 SH_C3[5] * z * (xx - yy), SH_C3[6] * x * (xx - 3 * yy)]
    return torch.stack(cols, dim=-1)


def fibonacci_dirs(normals: torch.Tensor, Ns: int, rand: torch.Tensor | None = None, pi: float = np.pi):
    """Fibonacci hemisphere directions around +z rotated onto each normal: [P, Ns, 3].
    `rand` [P, 1] in [0, 1) adds the training-time random rotation 2*pi*rand. Same data flow as
    fibonacci_sphere_sampling: a [P, 3, 3] rotation (z -> n, Rodrigues form with v = z x n)
    times the [.., 3, Ns] samples, normalised over the coordinate axis."""
    delta = pi * (3.0 - np.sqrt(5.0))
    i = torch.arange(Ns, dtype=torch.float32)[None]
    z = 1 - 2 * i / (2 * Ns - 1)
    rad = torch.sqrt(1 - z * z)
    theta = delta * i
    if rand is not None:
        theta = rand * 2 * pi + theta
    samples = torch.stack([torch.sin(theta) * rad, torch.cos(theta) * rad, z.expand_as(theta)], dim=-2)
    v1, v2 = -normals[..., 1], normals[..., 0]
    cp1 = (normals[..., 2] + 1).clamp_min(1e-7)
    zero = torch.zeros_like(v1)
    R = torch.stack([
        torch.stack([1 - v2 * v2 / cp1, v1 * v2 / cp1, v2], -1),
        torch.stack([v1 * v2 / cp1, 1 - v1 * v1 / cp1, -v1], -1),
        torch.stack([-v2, v1, 1 - (v1 * v1 + v2 * v2) / cp1 + zero], -1)], -2)   # [P, 3, 3]
    d = R @ samples                                                               # [P, 3, Ns]
    d = d / d.norm(dim=-2, keepdim=True).clamp_min(1e-12)
    return d.transpose(-1, -2)


def rendering_equation(base, rough, metal, normals, viewdirs, incidents, env, visibility, Ns: int = 24,
                       rand: torch.Tensor | None = None, pi: float = np.pi):
    """pbr [P,3] and the per-sample extras of rendering_equation_python (neilf.py:437-519), with
    the same tensor shapes per step ([P, Ns, 3, C] products summed over C, [P, Ns, 3] BRDF terms).
    incidents [P,S,3], env [1,S,3] (or None), visibility [P,S,1]; rand [P,1] for training."""
    P = base.shape[0]
    dirs = fibonacci_dirs(normals, Ns, rand, pi)                     # [P, Ns, 3]
    deg = int(round(np.sqrt(visibility.shape[1]))) - 1
    Y = sh_basis(deg, dirs).unsqueeze(2)                             # [P, Ns, 1, C]
    sh_local = incidents.transpose(1, 2).reshape(P, 1, 3, -1)        # [P, 1, 3, S]
    sh_vis = visibility.transpose(1, 2).reshape(P, 1, 1, -1)
    local = (Y[..., :sh_local.shape[-1]] * sh_local).sum(-1).clamp_min(0)
    if env is not None:
        sh_env = env.transpose(1, 2).unsqueeze(1)                    # [1, 1, 3, S]
        glob = ((Y[..., :sh_env.shape[-1]] * sh_env).sum(-1) + 0.5).clamp_min(0)
    else:
        glob = torch.zeros_like(local)
    vis = ((Y[..., :sh_vis.shape[-1]] * sh_vis).sum(-1) + 0.5).clamp(0, 1)
    glob = glob * vis
    light = local + glob
    b, r, m = base[:, None], rough[:, None], metal[:, None]
    n, v = normals[:, None], viewdirs[:, None]
    h = dirs + v
    h = h / h.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    hdn = (h * n).sum(-1, keepdim=True).clamp_min(0)
    hdo = (h * v).sum(-1, keepdim=True).clamp_min(0)
    ndi = (n * dirs).sum(-1, keepdim=True).clamp_min(0)
    ndo = (n * v).sum(-1, keepdim=True).clamp_min(0)
    f_d = (1 - m) * b / pi
    r2 = (r * r).clamp_min(1e-7)
    D = (1 / (r2 * pi)) * torch.exp((2 / r2) * (hdn - 1))
    F0 = 0.04 * (1 - m) + b * m
    Fr = F0 + (1.0 - F0) * (1.0 - hdo) ** 5
    k = (1 + r) ** 2 / 8
    V = (0.5 / (ndi * (1 - k) + k).clamp_min(1e-7)) * (0.5 / (ndo * (1 - k) + k).clamp_min(1e-7))
    f_s = D * Fr * V
    areas = torch.ones_like(dirs[..., :1]) * 2 * pi                  # incident area per sample
    transport = light * areas * ndi
    rgb_d = (f_d * transport).mean(-2)
    rgb_s = (f_s * transport).mean(-2)
    return rgb_d + rgb_s, dict(incident_dirs=dirs, incident_lights=light, local_incident_lights=local,
                               global_incident_lights=glob, incident_visibility=vis,
                               diffuse_light=transport.mean(-2))


def c1_inputs(P: int = 10_000, seed: int = 0):
    """SURVEY.md §8d config C1 inputs as torch CPU tensors."""
    rng = np.random.default_rng(seed)
    n = rng.normal(size=(P, 3)); n /= np.linalg.norm(n, axis=1, keepdims=True)
    v = rng.normal(size=(P, 3)); v /= np.linalg.norm(v, axis=1, keepdims=True)
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    return dict(base=f(rng.uniform(0, 1, (P, 3))), rough=f(rng.uniform(0.05, 1, (P, 1))),
                metal=f(rng.uniform(0, 1, (P, 1))), normals=f(n), viewdirs=f(v),
                incidents=f(rng.normal(0, 0.1, (P, 16, 3))), env=f(rng.normal(0, 0.1, (1, 16, 3))),
                visibility=f(rng.normal(0, 0.1, (P, 16, 1))))
