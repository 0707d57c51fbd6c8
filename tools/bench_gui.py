"""Timing of the GUI shader path (gui.py:464-467 -> forward.cu:805-1047) at M1 size on 1 GPU.

M1 scene (SURVEY.md §8d generator, 1M Gaussians, 1920x1080) with S = 21 feature channels (the
reference's 21-channel layout, which the feature-reading shaders and passes need), the reference's
own textures (tests/golden/textures.npz), and three forward variants:
  default   all-default shader managers (the fused default path, render_fwd_glds_kernel);
  shaders   every Gaussian in a non-default SH shader bucket and a non-default splat shader bucket
            (random ids, seed 0): working copies, sh_shader_kernel<ID> per bucket, the
            intermediate depth / stencil pass (intermediate_glds_kernel), splat_shader_kernel<ID> per
            bucket, shader_record_kernel, render_fwd_glds_kernel<SHADER=true>;
  gui       `shaders` + the post-process list [QuantizeLighting, SobelFilter, Invert].
Median of --iters forward calls after warmup, HIP events on the current stream. Run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.

Usage: python tools/bench_gui.py [--iters 10] [--P 1000000] [--out gpurun_out/gui.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SH_NAMES = ["CullHalf", "ExpPos", "GaussDissolve", "Heartbeat"]
SPLAT_NAMES = ["Crack", "CrackNoRecon", "Dissolve", "NaiveOutline", "QuantizeFlats", "QuantizeLight",
               "RoughnessOnly", "Stencil", "Wireframe"]
POST = ["QuantizeLighting", "SobelFilter", "Invert"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    import relightable3dgaussian_amd as r3
    from relightable3dgaussian_amd import synthetic

    _C = r3._C
    dev = torch.device("cuda", 0)
    T = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float32, device=dev)  # noqa: E731
    empty = torch.empty(0, device=dev)
    cam = synthetic.m1_camera(1920, 1080)
    scene = synthetic.m1_scene(P=a.P, S=21, seed=0, cam=cam)
    g = dict(means3D=T(scene.means3D), feats=T(scene.features), opac=T(scene.opacity), scales=T(scene.scales),
             rots=T(scene.rotations), sh=T(scene.sh))

    z = np.load(os.path.join(ROOT, "tests", "golden", "textures.npz"))
    handles = {}
    for name in z.files:
        pix = z[name].astype(np.float32) / np.float32(255.0)
        d = {"pixelData": torch.tensor(pix, device=dev),
             "height": torch.tensor([pix.shape[0]], dtype=torch.int32),
             "width": torch.tensor([pix.shape[1]], dtype=torch.int32),
             "encoding_mode": torch.tensor([_C.EncodeTextureMode("RGBA")], dtype=torch.int32),
             "wrap_modes": torch.tensor([_C.EncodeWrapMode("Wrap")] * 2, dtype=torch.int32),
             "normalizedCoords": torch.tensor([1], dtype=torch.int32)}
        handles[name] = _C.AllocateTexture(d)
    names = list(handles)
    texm = _C.UploadTexturesToDevice(names, [handles[n] for n in names], handles["Error"])
    rng = np.random.default_rng(0)
    shm, spm = _C.GetShShaderAddressMap(), _C.GetSplatShaderAddressMap()
    sh_ids = rng.integers(0, len(SH_NAMES), a.P)
    sp_ids = rng.integers(0, len(SPLAT_NAMES), a.P)
    sh_mgr = _C.create_shader_manager(0, torch.tensor([shm[SH_NAMES[i]] for i in sh_ids], dtype=torch.int64))
    sp_mgr = _C.create_shader_manager(1, torch.tensor([spm[SPLAT_NAMES[i]] for i in sp_ids], dtype=torch.int64))
    pp = _C.GetPostProcessShaderAddressMap()
    post = [pp[n] for n in POST]

    def fwd(sh=None, sp=None, passes=None):
        return _C.rasterize_gaussians(T([1.0, 1.0, 1.0]), 2500.0, 0.0, g["means3D"], g["feats"], empty, g["opac"],
                                      g["scales"], g["rots"], 1.0, empty, T(cam.view), T(cam.view_inv), T(cam.proj),
                                      T(cam.proj_inv), cam.tanfovx, cam.tanfovy, cam.cx, cam.cy, cam.height,
                                      cam.width, g["sh"], 3, T(cam.campos), False, True, texm, sh, sp, passes, False)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    res = {"config": f"M1 scene P={a.P}, 1920x1080, S=21, reference textures; SH ids U{{0..3}}, splat ids "
                     f"U{{non-default}}, post {POST}", "iters": a.iters}
    res["default_fwd_ms"] = round(timed(lambda: fwd()), 4)
    res["shaders_fwd_ms"] = round(timed(lambda: fwd(sh_mgr, sp_mgr)), 4)
    res["gui_fwd_ms"] = round(timed(lambda: fwd(sh_mgr, sp_mgr, post)), 4)
    res["shader_over_default"] = round(res["shaders_fwd_ms"] / res["default_fwd_ms"], 3)
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
