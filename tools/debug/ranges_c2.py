"""Debug: C2 tile ranges GPU vs oracle (prints mismatching tiles)."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import oracle
from relightable3dgaussian_amd import synthetic
import relightable3dgaussian_amd as r
from tests._helpers import hip_forward
from tests.test_gpu_parity import _oracle_fwd

cam = synthetic.orbit_camera(0.0, 30.0, 4.0311, 0.6911112, 800, 800)
scene = synthetic.ball_scene(300_000, S=21, seed=0)
h = hip_forward(r._C, scene, cam, S=21)
o = _oracle_fwd(scene, cam, 21)
L = h["num_rendered"]
st = r._C.rasterizer_state(h["geom"], h["binning"], h["image"], scene.P, cam.height, cam.width, L)
rg = st[2].cpu().numpy().view(np.uint32)
orr = o["ranges"]
bad = np.nonzero((rg != orr).any(1))[0]
print("L", L, "T", len(rg), "bad", len(bad))
for t in bad[:20]:
    print(t, rg[t], orr[t])
ts = (st[0].cpu().numpy().view(np.uint64) >> 32).astype(np.int64)
print("tile_sorted sorted:", bool(np.all(ts[1:] >= ts[:-1])), ts[:5], ts[-5:])
