"""Debug: is r3dg_sh_grad_from_views bitwise the per-view dL_dsh (one view, then two)?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import relightable3dgaussian_amd as r3  # noqa: E402
from relightable3dgaussian_amd import synthetic  # noqa: E402
from tests._helpers import hip_backward, hip_forward, tt, upstream_grads  # noqa: E402

_C = r3._C
scene = synthetic.ball_scene(20_000, S=21, seed=0)
P = scene.P
per, drgb, cams = [], [], []
for k in range(2):
    cam = synthetic.orbit_camera(45.0 * k, 30.0, 4.0311, 0.6911112, 200, 200)
    h = hip_forward(_C, scene, cam, S=21)
    dc, do, dd, df = upstream_grads(cam.height, cam.width, 21, seed=100 + k)
    g = hip_backward(_C, h, dc, do, dd, df)
    per.append(g["dL_dsh"])
    drgb.append(_C.sh_color_grads(h["geom"], P, tt(g["dL_dcolors"]), 0, P))
    cams.append(np.asarray(cam.campos, np.float32))
    for n in (1,):
        out = torch.full((P, 16, 3), float("nan"), device="cuda")
        _C.sh_grad_from_views(tt(scene.means3D), tt(cams[k][None]), drgb[k][None].contiguous(), 3, 0, out)
        o = out.cpu().numpy()
        ref = g["dL_dsh"]
        bad = o != ref
        print(f"view {k}: mismatched {bad.sum()} of {bad.size}; per coefficient:", bad.reshape(P, 16, 3).any(2).sum(0))
        if bad.any():
            i = np.argwhere(bad)[0]
            print("  first", i, o[tuple(i)], ref[tuple(i)], "drgb", drgb[k][i[0]].cpu().numpy(),
                  "dcol", g["dL_dcolors"][i[0]])
out = torch.full((P, 16, 3), float("nan"), device="cuda")
_C.sh_grad_from_views(tt(scene.means3D), tt(np.stack(cams)), torch.stack(drgb).contiguous(), 3, 0, out)
o = out.cpu().numpy()
ref = per[0] + per[1]
bad = o != ref
print(f"two views: mismatched {bad.sum()} of {bad.size}")
if bad.any():
    i = tuple(np.argwhere(bad)[0])
    print("  first", i, repr(o[i]), repr(ref[i]), repr(per[0][i]), repr(per[1][i]),
          "f32 sum", repr(np.float32(per[0][i]) + np.float32(per[1][i])))
