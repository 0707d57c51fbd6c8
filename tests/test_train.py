"""Training step on the device: oracle vs the reference's own GaussianModel
(tests/golden/train.npz, made by tests/golden/make_golden_train.py), the sharded optimizer's
exchange on CPU (gloo, world size 2), and on the GPU the HIP path (csrc/optim.hip through
relightable3dgaussian_amd.trainer) replaying the reference's sequence: 3 Adam steps with a
scheduled xyz learning rate, densification statistics, densify_and_prune (clone + split +
prune, with the stored split noise) and reset_opacity.

Tolerances: Adam / statistics / densify restate fp32 elementwise arithmetic, so they agree to a
few ulp (rtol 2e-5, atol 1e-6 -- parameters are O(1), steps O(lr)); the order of the densified
Gaussians and every copy is exact."""
from __future__ import annotations

import os
import socket
import types

import numpy as np
import pytest

from oracle import train_oracle as T

GOLD = os.path.join(os.path.dirname(__file__), "golden", "train.npz")
NAMES = [n for n, _ in T.GROUPS]
RTOL, ATOL = 2e-5, 1e-6


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _model(g, prefix):
    return {n: g[f"{prefix}_{n}"].astype(np.float32) for n in NAMES}


def _close(a, b, what):
    np.testing.assert_allclose(a, b, rtol=RTOL, atol=ATOL, err_msg=what)


def _opt_args():
    return types.SimpleNamespace(
        percent_dense=0.01, position_lr_init=0.00016, position_lr_final=0.0000016, position_lr_delay_mult=0.01,
        position_lr_max_steps=30000, normal_lr=0.01, rotation_lr=0.001, scaling_lr=0.005, opacity_lr=0.05,
        sh_lr=0.0025, base_color_lr=0.01, roughness_lr=0.01, metallic_lr=0.01, light_lr=0.002, light_rest_lr=-1.0,
        visibility_lr=0.0025, visibility_rest_lr=-1.0)


def test_fixture_exercises_clone_split_prune(gold):
    P0, Pn = gold["init_xyz"].shape[0], int(gold["P_densified"])
    assert Pn != P0
    assert np.isfinite(gold["densified_xyz"]).all()


def test_oracle_lr_schedule(gold):
    it0 = int(gold["iteration0"])
    for k in range(3):
        lr = T.expon_lr(it0 + k, 0.00016 * 2.5, 0.0000016 * 2.5, lr_delay_mult=0.01, max_steps=30000)
        np.testing.assert_allclose(gold[f"lr_{k}"][0], lr, rtol=1e-12)


def _oracle_sequence(g):
    model = _model(g, "init")
    m = {n: np.zeros_like(model[n]) for n in NAMES}
    v = {n: np.zeros_like(model[n]) for n in NAMES}
    P = model["xyz"].shape[0]
    acc, nacc, den, mr = (np.zeros(P, np.float32) for _ in range(4))
    for k in range(3):
        lrs = g[f"lr_{k}"]
        if k >= 1:
            T.densification_stats(g[f"means2D_grad{k}"], None, g[f"radii{k}"], acc, nacc, den, mr)
            # normal term: normalize(_normal.grad) of the step's gradient
            vis = g[f"radii{k}"] > 0
            ng = g[f"grad{k}_normal"][vis]
            u = ng / np.maximum(np.linalg.norm(ng, axis=-1, keepdims=True), np.float32(1e-3))
            nacc[vis] += np.linalg.norm(u, axis=-1).astype(np.float32)
        for gi, n in enumerate(NAMES):
            model[n], m[n], v[n] = T.adam_step(model[n], g[f"grad{k}_{n}"], m[n], v[n], lrs[gi], k + 1)
        yield k, model, m, v, (acc, nacc, den, mr)


def test_oracle_adam_and_stats_match_reference(gold):
    for k, model, m, v, stats in _oracle_sequence(gold):
        for n in NAMES:
            _close(model[n], gold[f"after{k}_{n}"], f"param {n} step {k}")
            _close(m[n], gold[f"after{k}_m_{n}"], f"exp_avg {n} step {k}")
            _close(v[n], gold[f"after{k}_v_{n}"], f"exp_avg_sq {n} step {k}")
    acc, nacc, den, mr = stats
    _close(acc, gold["xyz_accum"], "xyz_gradient_accum")
    _close(nacc, gold["normal_accum"], "normal_gradient_accum")
    np.testing.assert_array_equal(den, gold["denom"])
    np.testing.assert_array_equal(mr, gold["max_radii2D"])


def test_oracle_densify_and_reset_match_reference(gold):
    *_, (k, model, m, v, stats) = list(_oracle_sequence(gold))
    acc, nacc, den, mr = stats
    mg, mo, ext, mss, mgn, pd = gold["densify_args"]
    out, om, ov = T.densify_and_prune(model, m, v, acc, nacc, den, mr, mg, mo, ext, mss, mgn, pd, gold["noise"])
    assert out["xyz"].shape[0] == int(gold["P_densified"])
    for n in NAMES:
        _close(out[n], gold[f"densified_{n}"], f"densified {n}")
        _close(om[n], gold[f"densified_m_{n}"], f"densified exp_avg {n}")
        _close(ov[n], gold[f"densified_v_{n}"], f"densified exp_avg_sq {n}")
    T.reset_opacity(out, om, ov)
    for n in NAMES:
        _close(out[n], gold[f"reset_{n}"], f"reset {n}")
        _close(om[n], gold[f"reset_m_{n}"], f"reset exp_avg {n}")


# ---- sharded optimizer exchange (gloo, world size 2, CPU) ---------------------------------------

def _cpu_adam(P, widths, roles, param, g, m, v, lo, hi, lrs, b1, b2, eps, step):
    """The oracle standing in for _C.adam_step on CPU tensors (what is tested is the exchange)."""
    import torch

    bounds = np.cumsum([0] + [P * w for w in widths])
    gi = np.arange(lo, hi)
    lr = np.asarray(lrs, np.float64)[np.searchsorted(bounds, gi, side="right") - 1]
    p, mm, vv = T.adam_step(param[lo:hi].numpy(), g.numpy(), m.numpy(), v.numpy(), lr, step, b1, b2, eps)
    param[lo:hi] = torch.from_numpy(p)
    m.copy_(torch.from_numpy(mm))
    v.copy_(torch.from_numpy(vv))


def _tensors(g):
    import torch

    from relightable3dgaussian_amd import trainer

    shapes = dict(trainer.BASE_GROUPS + trainer.PBR_GROUPS)
    P = g["init_xyz"].shape[0]
    return {n: torch.from_numpy(g[f"init_{n}"]).reshape(P, *shapes[n]).contiguous() for n in NAMES}


def _shard_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from relightable3dgaussian_amd import trainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = dict(np.load(GOLD))
    st = trainer.GaussianTrainState.from_tensors(_tensors(g), world=world, rank=rank)
    st.training_setup(_opt_args(), spatial_lr_scale=2.5)
    for k in range(3):
        st.update_learning_rate(int(g["iteration0"]) + k)
        for n in NAMES:
            # each rank contributes half of the gradient: the reduce-scatter sums the views
            st.grad_view(n).copy_(torch.from_numpy(g[f"grad{k}_{n}"]).reshape(st.grad_view(n).shape) * 0.5)
        st.step(adam_fn=_cpu_adam)
    q.put((rank, {n: st.view(n).reshape(st.P, -1).numpy().copy() for n in NAMES}))
    dist.destroy_process_group()


def test_sharded_step_gloo_world2(gold):
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        for n in NAMES:
            # x * 0.5 + x * 0.5 == x exactly, so the sharded run must match the reference's steps
            _close(res[r][n], gold[f"after2_{n}"], f"rank {r} param {n}")


# ---- GPU: the HIP path replays the reference's sequence ----------------------------------------

@pytest.mark.gpu
def test_gpu_train_sequence_matches_reference(gold, hip_ext):
    import torch

    from relightable3dgaussian_amd import trainer

    dev = torch.device("cuda", 0)
    t = {n: x.to(dev) for n, x in _tensors(gold).items()}
    st = trainer.GaussianTrainState.from_tensors(t)
    st.training_setup(_opt_args(), spatial_lr_scale=2.5)
    P = st.P

    def flat(n, buf=None):
        return (buf if buf is not None else st.view(n)).reshape(P, -1).cpu().numpy()

    for k in range(3):
        st.update_learning_rate(int(gold["iteration0"]) + k)
        np.testing.assert_allclose(st.lrs, gold[f"lr_{k}"], rtol=1e-7)
        for n in NAMES:
            st.grad_view(n).copy_(torch.from_numpy(gold[f"grad{k}_{n}"]).reshape(st.grad_view(n).shape))
        if k >= 1:
            st.add_densification_stats(torch.from_numpy(gold[f"means2D_grad{k}"]).to(dev),
                                       torch.from_numpy(gold[f"radii{k}"]).to(dev),
                                       normal_grad=st.grad_view("normal").reshape(P, 3).clone())
        st.step()
        for n in NAMES:
            _close(flat(n), gold[f"after{k}_{n}"], f"param {n} step {k}")
        m = st._view(st.exp_avg, "normal").reshape(P, -1).cpu().numpy()
        _close(m, gold[f"after{k}_m_normal"], f"exp_avg normal step {k}")
    _close(st.xyz_gradient_accum.reshape(-1).cpu().numpy(), gold["xyz_accum"], "xyz_gradient_accum")
    _close(st.normal_gradient_accum.reshape(-1).cpu().numpy(), gold["normal_accum"], "normal_gradient_accum")
    np.testing.assert_array_equal(st.denom.reshape(-1).cpu().numpy(), gold["denom"])
    np.testing.assert_array_equal(st.max_radii2D.cpu().numpy(), gold["max_radii2D"])

    mg, mo, ext, mss, mgn, pd = gold["densify_args"]
    counts = st.densify_and_prune(mg, mo, ext, mss, mgn, noise=torch.from_numpy(gold["noise"]).to(dev))
    assert st.P == int(gold["P_densified"]), counts
    P = st.P
    for n in NAMES:
        _close(flat(n), gold[f"densified_{n}"], f"densified {n}")
        _close(st._view(st.exp_avg, n).reshape(P, -1).cpu().numpy(), gold[f"densified_m_{n}"], f"exp_avg {n}")
        _close(st._view(st.exp_avg_sq, n).reshape(P, -1).cpu().numpy(), gold[f"densified_v_{n}"], f"exp_avg_sq {n}")
    assert float(st.denom.abs().sum()) == 0.0  # densification_postfix
    st.reset_opacity()
    for n in ("opacity", "xyz"):
        _close(flat(n), gold[f"reset_{n}"], f"reset {n}")
    _close(st._view(st.exp_avg, "opacity").reshape(P, -1).cpu().numpy(), gold["reset_m_opacity"], "reset m")


@pytest.mark.gpu
def test_gpu_prune_only_and_adam_large(hip_ext):
    """`prune` keeps the survivors' statistics; Adam over a 1M-Gaussian flat buffer vs the oracle."""
    import torch

    from relightable3dgaussian_amd import trainer

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    P = 1 << 20
    shapes = dict(trainer.BASE_GROUPS + trainer.PBR_GROUPS)
    t = {n: torch.from_numpy(rng.normal(size=(P,) + shapes[n]).astype(np.float32)).to(dev) for n in NAMES}
    t["opacity"] = torch.from_numpy(rng.uniform(-7, 3, size=(P, 1)).astype(np.float32)).to(dev)
    t["scaling"] = torch.from_numpy(np.log(rng.uniform(0.002, 0.15, size=(P, 3))).astype(np.float32)).to(dev)
    st = trainer.GaussianTrainState.from_tensors(t)
    st.training_setup(_opt_args())
    g = torch.from_numpy((rng.normal(size=st.total()) * 1e-3).astype(np.float32)).to(dev)
    st.grad[:st.total()] = g
    p0 = st.param[:st.total()].cpu().numpy()
    st.step()
    bounds = np.cumsum([0] + [P * w for w in st.widths()])
    lr = np.asarray(st.lrs)[np.searchsorted(bounds, np.arange(st.total()), side="right") - 1]
    ref, _, _ = T.adam_step(p0, g.cpu().numpy(), np.zeros_like(p0), np.zeros_like(p0), lr, 1)
    np.testing.assert_allclose(st.param[:st.total()].cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    st.max_radii2D.copy_(torch.from_numpy(rng.uniform(0, 40, size=P).astype(np.float32)).to(dev))
    st.denom.fill_(3.0)
    op = st.view("opacity").cpu().numpy()[:, 0]
    keep_ref = ~((T._sigmoid(op) < np.float32(0.005)) | (st.max_radii2D.cpu().numpy() > np.float32(20.0))
                 | (np.exp(st.view("scaling").cpu().numpy()).max(1) > np.float32(0.1)))
    xyz_before = st.view("xyz").cpu().numpy()
    st.prune(0.005, 1.0, 20.0)
    assert 0 < st.P == int(keep_ref.sum()) < P
    np.testing.assert_array_equal(st.view("xyz").cpu().numpy(), xyz_before[keep_ref])
    assert float(st.denom.min()) == 3.0  # survivors keep their statistics


def _cpu_adam_groups(P, widths, roles, param, g, m, v, lo, hi, lrs, b1, b2, eps, steps):
    """Per-group oracle Adam: steps is one int (all groups) or one count per group, <= 0 = skip."""
    import torch

    steps = [steps] * len(widths) if np.isscalar(steps) else list(steps)
    bounds = np.cumsum([0] + [P * w for w in widths])
    for gi_, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        a, b = max(a, lo), min(b, hi)
        if a >= b or steps[gi_] <= 0:
            continue
        sl = slice(a - lo, b - lo)
        p, mm, vv = T.adam_step(param[a:b].numpy(), g[sl].numpy(), m[sl].numpy(), v[sl].numpy(), lrs[gi_],
                                steps[gi_], b1, b2, eps)
        param[a:b] = torch.from_numpy(p)
        m[sl] = torch.from_numpy(mm)
        v[sl] = torch.from_numpy(vv)


def _absent_sequence(st, adam_fn, dev):
    """Three steps; "normal" has no gradient in step 1 (grad None in the reference) and "opacity"
    is simply not written in step 2. Returns the per-step snapshots of both groups."""
    import torch

    rng = np.random.default_rng(7)
    snaps = []
    for k in range(3):
        for n, _ in st.groups:
            if (k == 1 and n == "normal") or (k == 2 and n == "opacity"):
                continue
            gv = st.grad_view(n)
            gv.copy_(torch.from_numpy(rng.normal(size=tuple(gv.shape)).astype(np.float32) * 1e-2).to(dev))
        st.step(adam_fn=adam_fn, absent=("normal",) if k == 1 else ())
        snaps.append({n: st.view(n).cpu().numpy().copy() for n in ("normal", "opacity", "xyz")})
        snaps[-1]["m_normal"] = st._view(st.exp_avg, "normal").cpu().numpy().copy()
    return snaps


def _check_absent(snaps, st):
    # step 1 skipped "normal": param and exp_avg unchanged across it
    np.testing.assert_array_equal(snaps[1]["normal"], snaps[0]["normal"])
    np.testing.assert_array_equal(snaps[1]["m_normal"], snaps[0]["m_normal"])
    assert st.group_steps[[n for n, _ in st.groups].index("normal")] == 2
    assert st.group_steps[[n for n, _ in st.groups].index("xyz")] == 3


def test_step_absent_and_unwritten_groups_cpu(gold):
    """the gradient buffer is cleared after every step by default (an unwritten group
    steps with a zero gradient, never the previous one), and `absent` groups are skipped as
    torch.optim.Adam skips a None grad (per-group step counts)."""
    import torch

    from relightable3dgaussian_amd import trainer

    st = trainer.GaussianTrainState.from_tensors(_tensors(gold))
    st.training_setup(_opt_args(), spatial_lr_scale=2.5)
    snaps = _absent_sequence(st, _cpu_adam_groups, torch.device("cpu"))
    _check_absent(snaps, st)
    assert float(st.grad.abs().sum()) == 0.0


@pytest.mark.gpu
def test_gpu_step_absent_matches_oracle(gold, hip_ext):
    """The HIP Adam (`adam_step_groups`) replays the same absent / unwritten sequence as the oracle."""
    import torch

    from relightable3dgaussian_amd import trainer

    dev = torch.device("cuda", 0)
    ref = trainer.GaussianTrainState.from_tensors(_tensors(gold))
    ref.training_setup(_opt_args(), spatial_lr_scale=2.5)
    want = _absent_sequence(ref, _cpu_adam_groups, torch.device("cpu"))
    st = trainer.GaussianTrainState.from_tensors({n: x.to(dev) for n, x in _tensors(gold).items()})
    st.training_setup(_opt_args(), spatial_lr_scale=2.5)
    got = _absent_sequence(st, None, dev)
    _check_absent(got, st)
    for k in range(3):
        for n in want[k]:
            _close(got[k][n].reshape(st.P, -1), want[k][n].reshape(st.P, -1), f"step {k} {n}")


def test_absent_group_matches_torch_adam_cpu(gold):
    """the `absent` semantics against torch.optim.Adam itself (single-tensor, CPU), not a
    hand-written Adam: two steps, every group with a gradient in the first, "normal" with
    grad=None in the second. param, exp_avg, exp_avg_sq and state['step'] per group must equal the
    trainer's (CPU Adam of oracle/train_oracle.py, per-group step counts): step counts exactly,
    values to a few ulp (torch fuses its multiply-adds), and the absent group's param / exp_avg /
    exp_avg_sq untouched by the step it skipped, bit for bit in both."""
    import torch

    from relightable3dgaussian_amd import trainer

    tens = _tensors(gold)
    st = trainer.GaussianTrainState.from_tensors(tens)
    st.training_setup(_opt_args(), spatial_lr_scale=2.5)
    names = [n for n, _ in st.groups]
    params = {n: torch.nn.Parameter(st.view(n).clone()) for n in names}
    opt = torch.optim.Adam([{"params": [params[n]], "lr": lr, "name": n} for n, lr in zip(names, st.lrs)],
                           lr=0.0, eps=1e-15, foreach=False)
    rng = np.random.default_rng(11)
    kept = {}
    for k in range(2):
        if k == 1:
            kept = {"p": st.view("normal").clone(), "m": st._view(st.exp_avg, "normal").clone(),
                    "v": st._view(st.exp_avg_sq, "normal").clone(), "tp": params["normal"].detach().clone(),
                    "tm": opt.state[params["normal"]]["exp_avg"].clone()}
        for n in names:
            g = torch.from_numpy(rng.normal(size=tuple(params[n].shape)).astype(np.float32) * 1e-2)
            if k == 1 and n == "normal":
                params[n].grad = None
                continue
            params[n].grad = g.clone()
            st.grad_view(n).copy_(g)
        opt.step()
        st.step(adam_fn=_cpu_adam_groups, absent=("normal",) if k == 1 else ())
    for i, n in enumerate(names):
        s = opt.state[params[n]]
        # torch's CPU lerp / addcdiv fuse their multiply-adds (one rounding fewer than the oracle's
        # statements): values agree to a few ulp; the step counts exactly
        np.testing.assert_allclose(st.view(n).numpy(), params[n].detach().numpy(), rtol=1e-6, atol=1e-9, err_msg=n)
        for mine, ref in ((st._view(st.exp_avg, n), s["exp_avg"]), (st._view(st.exp_avg_sq, n), s["exp_avg_sq"])):
            np.testing.assert_allclose(mine.numpy(), ref.numpy(), rtol=1e-6, atol=1e-6 * float(ref.abs().max()),
                                       err_msg=n)
        assert st.group_steps[i] == int(s["step"]), n
    assert st.group_steps[names.index("normal")] == 1 and st.group_steps[names.index("xyz")] == 2
    assert torch.equal(st.view("normal"), kept["p"]) and torch.equal(st._view(st.exp_avg, "normal"), kept["m"])
    assert torch.equal(st._view(st.exp_avg_sq, "normal"), kept["v"])
    assert torch.equal(params["normal"].detach(), kept["tp"])
    assert torch.equal(opt.state[params["normal"]]["exp_avg"], kept["tm"])
