"""Golden vectors for the Gaussian PLY format from the REFERENCE's own save_ply (CPU container).

Runs `GaussianModel.save_ply` (scene/gaussian_model.py:658-686, neilf model, SH degree 3) on
seeded parameters and records the structured vertex array it hands to `plyfile` (absent from
this image: `PlyElement.describe` / `PlyData.write` are replaced by recorders that only capture
their argument -- nothing of plyfile's own behaviour is restated here). The fixture holds, per
property, the reference's name order (`construct_list_of_attributes`, :630-656) and the float32
values, i.e. exactly the bytes plyfile writes after its `property float <name>` header.

  ply.npz   names [n], values [P, n] f32, and the parameters (trainer group names) that produced them

Usage:  python tests/golden/make_golden_ply.py  [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import CpuMode  # noqa: E402
from make_golden_train import GROUPS, load_gaussian_model  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    GaussianModel = load_gaussian_model(a.reference)
    captured = {}

    class PlyElement:
        @staticmethod
        def describe(elements, name):
            captured["elements"] = elements.copy()
            captured["name"] = name
            return elements

    class PlyData:
        def __init__(self, els):
            pass

        def write(self, path):
            captured["path"] = path

    g = GaussianModel.save_ply.__globals__  # the reference module's namespace
    g["PlyElement"], g["PlyData"] = PlyElement, PlyData
    rng = np.random.default_rng(11)
    P = 64
    out = {}
    with CpuMode():
        m = GaussianModel(3, render_type="neilf")
        for name, attr, shp in GROUPS:
            v = rng.normal(size=(P,) + shp).astype(np.float32)
            setattr(m, attr, torch.nn.Parameter(torch.tensor(v)))
            out[f"param_{name}"] = v
        with tempfile.TemporaryDirectory() as d:
            m.save_ply(os.path.join(d, "point_cloud.ply"))
    el = captured["elements"]
    assert captured["name"] == "vertex"
    names = list(el.dtype.names)
    out["names"] = np.array(names)
    out["values"] = np.stack([np.asarray(el[n], np.float32) for n in names], axis=1)
    np.savez_compressed(os.path.join(HERE, "ply.npz"), **out)
    print("wrote ply.npz", out["values"].shape)


if __name__ == "__main__":
    main()
