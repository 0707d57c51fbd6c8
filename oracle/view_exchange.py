"""CPU oracle -- TEST INFRASTRUCTURE ONLY (never imported by the product package).

numpy restatement of the view-parallel SH-gradient rebuild (include/r3dg_hip.h
r3dg_sh_color_grads / r3dg_sh_grad_from_views): the SH part of one view's gradient is rank 1 per
Gaussian, dL/dsh[k][c] = Y_k(dir) * dRGB[c] with dir = normalize(mean - campos) and dRGB the
colour gradient with the channels whose SH colour was clamped at 0 zeroed -- the SH lines of
computeColorFromSH's backward (reference r3dg-rasterization/cuda_rasterizer/backward.cu:20-139;
the basis constants are auxiliary.h:22-39). Pinned by tests/test_view_parallel.py against the sum
over views of the C oracle's own per-view dL_dsh (oracle/r3dg_oracle.c, rasterize_backward).
"""
from __future__ import annotations

import numpy as np

F = np.float32
C0 = F(0.28209479177387814)
C1 = F(0.4886025119029199)
C2 = [F(1.0925484305920792), F(-1.0925484305920792), F(0.31539156525252005), F(-1.0925484305920792),
      F(0.5462742152960396)]
C3 = [F(-0.5900435899266435), F(2.890611442640554), F(-0.4570457994644658), F(0.3731763325901154),
      F(-0.4570457994644658), F(1.445305721320277), F(-0.5900435899266435)]


def sh_basis(means3D, campos):
    """[P,16] SH basis of normalize(mean - campos) as backward.cu:27-57 evaluates it (float32)."""
    d = np.asarray(means3D, F) - np.asarray(campos, F)[None, :]
    ln = np.sqrt((d * d).sum(1, dtype=F)).astype(F)
    x, y, z = (d / ln[:, None]).T
    xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
    b = np.empty((d.shape[0], 16), F)
    b[:, 0] = C0
    b[:, 1], b[:, 2], b[:, 3] = -C1 * y, C1 * z, -C1 * x
    b[:, 4], b[:, 5] = C2[0] * xy, C2[1] * yz
    b[:, 6] = C2[2] * (F(2) * zz - xx - yy)
    b[:, 7], b[:, 8] = C2[3] * xz, C2[4] * (xx - yy)
    b[:, 9] = C3[0] * y * (F(3) * xx - yy)
    b[:, 10] = C3[1] * xy * z
    b[:, 11] = C3[2] * y * (F(4) * zz - xx - yy)
    b[:, 12] = C3[3] * z * (F(2) * zz - F(3) * xx - F(3) * yy)
    b[:, 13] = C3[4] * x * (F(4) * zz - xx - yy)
    b[:, 14] = C3[5] * z * (xx - yy)
    b[:, 15] = C3[6] * x * (xx - F(3) * yy)
    return b


def sh_color_grads(dL_dcolors, clamped):
    """dRGB: dL_dcolors [P,3] with channel c zeroed where bit c of clamped [P] is set."""
    mask = ((np.asarray(clamped, np.uint8)[:, None] >> np.arange(3, dtype=np.uint8)) & 1) == 0
    return np.where(mask, np.asarray(dL_dcolors, F), F(0))


def sh_grad_from_views(means3D, campos, drgb, degree, M):
    """sum over views v (in order) of Y_k(normalize(mean - campos[v])) * drgb[v][:, c]; [P,M,3]."""
    ncoef = (degree + 1) ** 2
    P = np.asarray(means3D).shape[0]
    out = np.zeros((P, M, 3), F)
    for v in range(len(campos)):
        b = sh_basis(means3D, campos[v])[:, :ncoef]
        out[:, :ncoef, :] += b[:, :, None] * np.asarray(drgb[v], F)[:, None, :]
    return out
