"""Lane utilisation of the blends' visit lists, and what finer lists would save.

    python tools/analysis/half_lists.py W H P [TILE_STRIDE]
    (M1: 1920 1080 1000000 9 -- every 9th tile, ~10 min on one core)

Model, from the oracle's binning and forward (CPU only; no GPU): a wave (8x8 quadrant) visits an
instance when one of its pixels blends it (the backward's exact visit list: alpha test passed and
position < n_contrib); "fwd" counts positions up to each pixel's stop instead (the forward's
evaluations, ignoring the conservative cull's extra). For visit lists per half (top / bottom 8x4,
"tb"; left / right 4x8, "lr") or per 4x4 quarter ("q4"), a wave's iterations are the longest of its
sub-lists and its reduction rows the sum of them. Prints both as fractions of today's visits.
Measured at M1: 24.9 blending lanes per visit; halves 0.833 of the iterations with 1.58x the rows,
quarters 0.70 with 2.52x."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", ".."))
import oracle  # noqa: E402
from relightable3dgaussian_amd import synthetic  # noqa: E402


def main():
    W, H, P = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    stride = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    cam = synthetic.m1_camera(W, H)
    scene = synthetic.m1_scene(P=P, S=3, seed=4, cam=cam)
    o = oracle.rasterize_forward(cam, scene.means3D, scene.opacity, scene.features, sh=scene.sh, scales=scene.scales,
                                 rotations=scene.rotations)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    pl, rg, m2, co = o["point_list"], o["ranges"], o["means2D"], o["conic_opacity"]
    nc = o["n_contrib"].reshape(H, W)
    stats = {k: [0, 0] for k in ["bwd_tb", "bwd_lr", "bwd_q4", "fwd_tb", "fwd_lr", "fwd_q4"]}
    visits = {"bwd": 0, "fwd": 0}
    lanes_ok = 0
    for t in range(0, gx * gy, stride):
        a, b = rg[t]
        if b <= a:
            continue
        ids = pl[a:b]
        tx, ty = t % gx, t // gx
        ys, xs = np.mgrid[ty * 16:ty * 16 + 16, tx * 16:tx * 16 + 16]
        ins = (xs < W) & (ys < H)
        px, py = xs.reshape(-1).astype(np.float32), ys.reshape(-1).astype(np.float32)
        c, mx = co[ids], m2[ids]
        dx, dy = mx[:, 0:1] - px[None], mx[:, 1:2] - py[None]
        power = (-0.5 * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy).astype(np.float32)
        alpha = np.minimum(0.99, c[:, 3:4] * np.exp(power))
        aok = (power <= 0) & (alpha >= 1 / 255.0) & ins.reshape(-1)[None]
        ncl = np.where(ins, nc[np.minimum(ys, H - 1), np.minimum(xs, W - 1)], 0).reshape(-1)
        pos = np.arange(b - a)[:, None]
        ok = aok & (pos < ncl[None])
        lanes_ok += int(ok.sum())
        fok = aok & (pos <= ncl[None])
        lx, ly = xs.reshape(-1) - tx * 16, ys.reshape(-1) - ty * 16
        for qd in range(4):
            qx, qy = (qd & 1) * 8, (qd >> 1) * 8
            inq = (lx >= qx) & (lx < qx + 8) & (ly >= qy) & (ly < qy + 8)
            parts = {"tb": [inq & (ly < qy + 4), inq & (ly >= qy + 4)],
                     "lr": [inq & (lx < qx + 4), inq & (lx >= qx + 4)],
                     "q4": [inq & (lx >= qx + 4 * (i & 1)) & (lx < qx + 4 * (i & 1) + 4) & (ly >= qy + 4 * (i >> 1))
                            & (ly < qy + 4 * (i >> 1) + 4) for i in range(4)]}
            for name, okm in (("bwd", ok), ("fwd", fok)):
                visits[name] += int(okm[:, inq].any(1).sum())
                for split, masks in parts.items():
                    n = [int(okm[:, m].any(1).sum()) for m in masks]
                    stats[f"{name}_{split}"][0] += max(n)
                    stats[f"{name}_{split}"][1] += sum(n)
    print("L", o["num_rendered"], "visits", visits, "blending lanes per visit", round(lanes_ok / visits["bwd"], 2))
    for k, (it, rows) in stats.items():
        base = visits[k[:3]]
        print(k, "iterations", round(it / base, 3), "rows", round(rows / base, 3))


if __name__ == "__main__":
    main()
