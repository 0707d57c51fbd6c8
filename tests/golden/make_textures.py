"""Writes tests/golden/textures.npz: the reference's own texture images (textures/*.png, loaded by
asset_processing/textureImport.py:13-43 under the names of its initialize_all_textures) as
RGBA uint8, decimated 4x to 128x128 to keep the fixture small. Data only -- run here, where
/root/reference exists; the GPU box reads the committed .npz.

    python tests/golden/make_textures.py
"""
import os

import numpy as np
from PIL import Image

SRC = "/root/reference/textures"
FILES = {"Cracks": "Cracks 2.png", "Turbulence": "Turbulence 2.png", "Craters": "Craters 12.png",
         "Depth cracks": "Depth Cracks.png", "Bulge": "bulge.png", "shadow": "shadow.png", "Error": "Error.png"}

out = {}
for name, f in FILES.items():
    im = Image.open(os.path.join(SRC, f))
    assert im.mode == "RGBA", (f, im.mode)
    a = np.asarray(im, dtype=np.uint8)[::4, ::4]
    out[name] = np.ascontiguousarray(a)
np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "textures.npz"), **out)
print({k: v.shape for k, v in out.items()})
