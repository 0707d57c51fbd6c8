"""Timing of the render-equation kernels on the GPU.

P Gaussians (default 1M), Ns = 24, S_inc = S_dir = S_vis = 16, inputs from synthetic.brdf_inputs.
Reports device time per call (HIP events on the current stream, median of K) and the effective
HBM rate against SURVEY.md §8d's per-Gaussian bytes: forward (training, with rand) 396 read +
312 written + 96 rand; complex forward 204 + 1312; backward 612 + 300.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch

    import relightable3dgaussian_amd as r
    from relightable3dgaussian_amd import synthetic

    _C = r._C
    inp = synthetic.brdf_inputs(args.P, seed=0)
    t = {k: torch.as_tensor(v, device="cuda") for k, v in inp.items()}
    ins = [t[k] for k in ["base", "rough", "metal", "normals", "viewdirs", "incidents", "env", "visibility"]]
    rnd = torch.rand(args.P, 24, 1, device="cuda")
    gp = torch.randn(args.P, 3, device="cuda")
    gd = torch.randn(args.P, 3, device="cuda")

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    dirs = _C.render_equation_forward(*ins, 24, False, False)[1]
    res = {}
    for name, fn, nbytes in [
        ("forward_train", lambda: _C.render_equation_forward_with_rand(*ins, 24, True, rnd), 396 + 312 + 96),
        ("forward_eval", lambda: _C.render_equation_forward(*ins, 24, False, False), 396 + 312),
        ("forward_complex", lambda: _C.render_equation_forward_complex(*ins, 24), 204 + 1312),
        ("backward", lambda: _C.render_equation_backward(*ins, 24, dirs, gp, gd, False), 612 + 300),
    ]:
        ms = timed(fn)
        res[name] = {"ms": round(ms, 4), "GB/s": round(nbytes * args.P / ms / 1e6, 1),
                     "Mgauss/s": round(args.P / ms / 1e3, 1)}
    print(json.dumps({"P": args.P, "Ns": 24, "results": res, "hbm_peak_GBs": 8000}))


if __name__ == "__main__":
    main()
