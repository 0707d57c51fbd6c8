"""Timing of the training step on the device, 1 GPU.

  * `_C.adam_step` over the full NeILF model (14 groups, 131 floats per Gaussian) at P Gaussians,
    against its HBM roofline: 28 algorithmic bytes per float (p, g, m, v read; p, m, v written);
  * beside it torch.optim.Adam -- the optimizer the reference calls (gaussian_model.py:613,
    eps=1e-15, 14 param groups; foreach path on the device) -- on the same tensors and GPU;
  * `densify_and_prune` (classification + scan + scatter of every group and both Adam states)
    with ~10 % of the Gaussians selected for clone / split.
Writes one JSON object (stdout and --out).

Usage: python tools/bench_train.py [--P 1000000] [--iters 20] [--out profiles/r01_train_timing.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from relightable3dgaussian_amd import trainer

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    P = a.P
    shapes = dict(trainer.BASE_GROUPS + trainer.PBR_GROUPS)
    t = {n: torch.from_numpy(rng.normal(size=(P,) + s).astype(np.float32)).to(dev) for n, s in shapes.items()}
    t["scaling"] = torch.from_numpy(np.log(rng.uniform(0.002, 0.03, size=(P, 3))).astype(np.float32)).to(dev)
    t["opacity"] = torch.from_numpy(rng.uniform(-4, 3, size=(P, 1)).astype(np.float32)).to(dev)
    st = trainer.GaussianTrainState.from_tensors(t)
    import types

    st.training_setup(types.SimpleNamespace(
        percent_dense=0.01, position_lr_init=0.00016, position_lr_final=0.0000016, position_lr_delay_mult=0.01,
        position_lr_max_steps=30000, normal_lr=0.01, rotation_lr=0.001, scaling_lr=0.005, opacity_lr=0.05,
        sh_lr=0.0025, base_color_lr=0.01, roughness_lr=0.01, metallic_lr=0.01, light_lr=0.002, light_rest_lr=-1.0,
        visibility_lr=0.0025, visibility_rest_lr=-1.0))
    n = st.total()
    st.grad[:n] = torch.randn(n, device=dev) * 1e-3

    def timed(fn, iters):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    def hip_step():
        from relightable3dgaussian_amd import _C

        st.step_count += 1
        _C.adam_step(st.P, st.widths(), st.roles(), st.param, st.grad[:n], st.exp_avg[:n], st.exp_avg_sq[:n], 0, n,
                     list(st.lrs), 0.9, 0.999, 1e-15, st.step_count)

    hip_ms = timed(hip_step, a.iters)
    bytes_ = 28.0 * n
    # torch.optim.Adam (foreach) on the reference's 14 separate parameters
    params = [torch.nn.Parameter(st.view(nm).clone()) for nm, _ in st.groups]
    for p, (nm, _) in zip(params, st.groups):
        p.grad = st.grad_view(nm).clone()
    opt = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(params, st.lrs)], lr=0.0, eps=1e-15)
    torch_ms = timed(opt.step, a.iters)
    # densify_and_prune with ~10 % selected
    sel = torch.rand(P, device=dev) < 0.1
    st.xyz_gradient_accum.copy_((sel.float() * 1e-3).reshape(P, 1))
    st.denom.fill_(1.0)
    snap = (st.param.clone(), st.exp_avg.clone(), st.exp_avg_sq.clone(), st.P)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    counts = st.densify_and_prune(2e-4, 0.005, 1.0, 20.0, 10.0)
    e1.record()
    torch.cuda.synchronize()
    dens_ms = e0.elapsed_time(e1)
    res = {
        "P": P, "floats_per_gaussian": sum(st.widths()), "groups": len(st.groups),
        "adam": {"hip_ms": round(hip_ms, 4), "algorithmic_bytes": bytes_, "achieved_GBps": round(bytes_ / hip_ms / 1e6, 1),
                 "peak_GBps": 8000.0, "frac": round(bytes_ / hip_ms / 1e6 / 8000.0, 4),
                 "torch_optim_adam_ms": round(torch_ms, 4), "speedup_vs_torch": round(torch_ms / hip_ms, 2)},
        "densify_and_prune": {"ms": round(dens_ms, 3), "P_before": snap[3], "P_after": st.P, "counts": counts},
    }
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
