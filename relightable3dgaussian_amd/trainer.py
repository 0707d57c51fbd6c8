"""Training step on the device around the rasterizer.

Mirrors the training-side API of the reference's GaussianModel (scene/gaussian_model.py:581-620
training_setup / step / update_learning_rate, :688-691 reset_opacity, :822-1062 prune_points,
densify_and_clone, densify_and_split, densify_and_prune, prune, add_densification_stats) and the
densification block of train.py:170-193 -- same method names and argument meaning -- over ONE
flat fp32 parameter buffer per model (group g = a [P, width_g] block, include/r3dg_hip.h
"training step on the device"), stepped by the HIP kernels of csrc/optim.hip through `_C`.

Multi-GPU (view-parallel training, one camera per rank per step): instead of
all-reducing the gradient bucket and stepping a full Adam on every rank, the optimizer is
sharded ZeRO-style: gradients are reduce-scattered (sum over views) so rank r owns the contiguous
flat range [r*S, (r+1)*S), Adam runs on that shard only with the shard's exp_avg / exp_avg_sq
(1/N of the optimizer memory), and the updated parameters are all-gathered. Reduce-scatter +
all-gather move the same bytes as one all-reduce, and the Adam work and state shrink N-fold.
Densification statistics are summed (accumulators, denom) / maxed (max_radii2D) over ranks at
densification time; rank 0 densifies and broadcasts the new model so every rank holds the same
Gaussians (the split noise is drawn once).

No CPU fallback: every kernel call goes through `_C`, which refuses non-device tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# scene/gaussian_model.py:586-612 Adam groups (use_pbr adds the last seven): name, shape per
# Gaussian (the reference's tensor shape without the leading P)
BASE_GROUPS = [("xyz", (3,)), ("normal", (3,)), ("rotation", (4,)), ("scaling", (3,)), ("opacity", (1,)),
               ("f_dc", (1, 3)), ("f_rest", (15, 3))]
PBR_GROUPS = [("base_color", (3,)), ("roughness", (1,)), ("metallic", (1,)), ("incidents_dc", (1, 3)),
              ("incidents_rest", (15, 3)), ("visibility_dc", (1, 1)), ("visibility_rest", (15, 1))]


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:30-66 (host-side scalar schedule, as the reference)."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        return delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)

    return helper


@dataclass
class _Dist:
    world: int = 1
    rank: int = 0
    group: object = None


@dataclass
class GaussianTrainState:
    """One model's parameters + Adam state + densification statistics on the device.

    `groups` is [(name, shape)] in Adam group order; `param` is the flat buffer (capacity padded to
    a multiple of 4 * world so every rank's shard is float4-aligned and equal-sized)."""

    groups: list
    P: int
    param: object                      # torch float32 [cap]
    grad: object                       # torch float32 [cap] (filled by the caller / views)
    exp_avg: object                    # [shard] (rank-local)
    exp_avg_sq: object
    lrs: list = field(default_factory=list)
    step_count: int = 0
    percent_dense: float = 0.0
    xyz_gradient_accum: object = None  # [P, 1]
    normal_gradient_accum: object = None
    denom: object = None
    max_radii2D: object = None         # [P]
    xyz_scheduler_args: object = None
    dist: _Dist = field(default_factory=_Dist)
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-15                 # gaussian_model.py:613

    # ---- construction ------------------------------------------------------------------------
    @staticmethod
    def from_tensors(tensors: dict, use_pbr: bool = True, world: int = 1, rank: int = 0, group=None):
        """tensors: name -> [P, *shape] (the reference's _xyz, _normal, ... values)."""
        import torch

        groups = BASE_GROUPS + (PBR_GROUPS if use_pbr else [])
        P = int(tensors["xyz"].shape[0])
        dev = tensors["xyz"].device
        st = GaussianTrainState(groups=groups, P=P, param=None, grad=None, exp_avg=None, exp_avg_sq=None,
                                dist=_Dist(world, rank, group))
        flat = torch.cat([tensors[n].reshape(-1).to(torch.float32) for n, _ in groups]) if P \
            else torch.zeros(0, device=dev)
        st._set_flat(flat, torch.zeros(st.shard_size(), device=dev), torch.zeros(st.shard_size(), device=dev),
                     keep_shard=True)
        st._reset_stats()
        return st

    def widths(self):
        # the group layout never changes after construction (densification changes P only):
        # computed once, so a step's host work stays small beside its ~0.2 ms kernel
        w = getattr(self, "_widths", None)
        if w is None:
            w = self._widths = [int(np.prod(s)) for _, s in self.groups]
        return w

    def roles(self):
        r = getattr(self, "_roles", None)
        if r is None:
            names = [n for n, _ in self.groups]
            r = self._roles = [names.index("xyz"), names.index("scaling"), names.index("rotation"),
                               names.index("opacity")]
        return r

    def total(self):
        return self.P * sum(self.widths())

    def shard_size(self):
        w = self.dist.world
        return int(math.ceil(max(self.total(), 1) / (4 * w)) * 4)

    def shard_range(self):
        s = self.shard_size()
        lo = min(self.dist.rank * s, self.total())
        return lo, min(lo + s, self.total())

    def _set_flat(self, flat, m_shard, v_shard, keep_shard=False):
        import torch

        cap = self.shard_size() * self.dist.world
        self.param = torch.zeros(cap, device=flat.device)
        self.param[:flat.numel()] = flat
        self.grad = torch.zeros(cap, device=flat.device)
        self.exp_avg, self.exp_avg_sq = m_shard, v_shard

    def _reset_stats(self):
        import torch

        dev = self.param.device
        self.xyz_gradient_accum = torch.zeros((self.P, 1), device=dev)
        self.normal_gradient_accum = torch.zeros((self.P, 1), device=dev)
        self.denom = torch.zeros((self.P, 1), device=dev)
        self.max_radii2D = torch.zeros((self.P,), device=dev)

    # ---- views (the reference's per-group tensors) -------------------------------------------
    def _view(self, buf, name):
        o = 0
        for n, s in self.groups:
            w = int(np.prod(s))
            if n == name:
                return buf[o:o + self.P * w].view(self.P, *s)
            o += self.P * w
        raise KeyError(name)

    def view(self, name):
        """The parameter tensor the reference calls `_<name>` (a view into the flat buffer)."""
        return self._view(self.param, name)

    def grad_view(self, name):
        return self._view(self.grad, name)

    # ---- gaussian_model.py:658-793 (PLY checkpoints) -------------------------------------------
    @staticmethod
    def load_ply(path: str, device="cuda", use_pbr: bool = True, max_sh_degree: int = 3, **kw):
        """load_ply (gaussian_model.py:693-793) straight into the flat parameter buffer."""
        import torch

        from .ply import load_ply

        arrs = load_ply(path, max_sh_degree=max_sh_degree, use_pbr=use_pbr)
        return GaussianTrainState.from_tensors({k: torch.from_numpy(v).to(device) for k, v in arrs.items()},
                                               use_pbr=use_pbr, **kw)

    def save_ply(self, path: str) -> None:
        """save_ply (gaussian_model.py:658-686) from the flat parameter buffer."""
        from .ply import save_ply

        names = [n for n, _ in self.groups]
        save_ply(path, {n: self.view(n) for n in names}, use_pbr="base_color" in names)

    # ---- gaussian_model.py:581-620 -------------------------------------------------------------
    def training_setup(self, training_args, spatial_lr_scale=1.0):
        a = training_args
        self.percent_dense = a.percent_dense
        self._reset_stats()
        lr = {"xyz": a.position_lr_init * spatial_lr_scale, "normal": a.normal_lr, "rotation": a.rotation_lr,
              "scaling": a.scaling_lr, "opacity": a.opacity_lr, "f_dc": a.sh_lr, "f_rest": a.sh_lr / 20.0}
        if any(n == "base_color" for n, _ in self.groups):
            light_rest = a.light_rest_lr if a.light_rest_lr >= 0 else a.light_lr / 20.0
            vis_rest = a.visibility_rest_lr if a.visibility_rest_lr >= 0 else a.visibility_lr / 20.0
            lr.update({"base_color": a.base_color_lr, "roughness": a.roughness_lr, "metallic": a.metallic_lr,
                       "incidents_dc": a.light_lr, "incidents_rest": light_rest, "visibility_dc": a.visibility_lr,
                       "visibility_rest": vis_rest})
        self.lrs = [float(lr[n]) for n, _ in self.groups]
        self.xyz_scheduler_args = get_expon_lr_func(lr_init=a.position_lr_init * spatial_lr_scale,
                                                    lr_final=a.position_lr_final * spatial_lr_scale,
                                                    lr_delay_mult=a.position_lr_delay_mult,
                                                    max_steps=a.position_lr_max_steps)

    def update_learning_rate(self, iteration):
        lr = self.xyz_scheduler_args(iteration)
        self.lrs[[n for n, _ in self.groups].index("xyz")] = float(lr)
        return lr

    def step(self, adam_fn=None, zero_grad: bool = True, absent=()):
        """optimizer.step() + zero_grad(set_to_none=True) (gaussian_model.py:615-617); sharded over
        ranks. `absent` names the groups whose gradient is None this iteration: torch.optim.Adam
        skips them (param, exp_avg, exp_avg_sq and the group's step count stay as they are), so
        they are skipped here too (per-group step counts, `_C.adam_step_groups`). The gradient
        buffer is cleared after the step (zero_grad=True, the default), so a group the caller does
        not write before the next step contributes a zero gradient, never the previous one; pass
        zero_grad=False only when every group is rewritten each step."""
        import torch.distributed as dist

        from . import _C

        names = [n for n, _ in self.groups]
        bad = set(absent) - set(names)
        if bad:
            raise KeyError(f"step: unknown groups {sorted(bad)}")
        gs = getattr(self, "group_steps", None)
        if gs is None or len(gs) != len(names):
            gs = self.group_steps = [self.step_count] * len(names)
        self.step_count += 1
        steps = []
        for i, n in enumerate(names):
            if n in absent:
                steps.append(0)
            else:
                gs[i] += 1
                steps.append(gs[i])
        lo, hi = self.shard_range()
        s = self.shard_size()
        if self.dist.world > 1:
            g = self.grad.new_empty(s)
            dist.reduce_scatter_tensor(g, self.grad, op=dist.ReduceOp.SUM, group=self.dist.group)
            g = g[:hi - lo]
        else:
            g = self.grad[lo:hi]
        args = (self.P, self.widths(), self.roles(), self.param, g.contiguous(), self.exp_avg[:hi - lo],
                self.exp_avg_sq[:hi - lo], lo, hi, list(self.lrs), self.betas[0], self.betas[1], self.eps)
        uniform = len(set(steps)) == 1 and steps[0] > 0
        if adam_fn is not None:
            adam_fn(*args, steps[0] if uniform else steps)
        elif uniform:
            _C.adam_step(*args, steps[0])
        else:
            _C.adam_step_groups(*args, steps)
        if self.dist.world > 1:
            dist.all_gather_into_tensor(self.param, self.param[self.dist.rank * s:(self.dist.rank + 1) * s].clone(),
                                        group=self.dist.group)
        if zero_grad:
            self.grad.zero_()

    # ---- densification (train.py:170-186, gaussian_model.py:1025-1062) ------------------------
    def add_densification_stats(self, dL_dmeans2D, radii, normal_grad=None):
        """max_radii2D update (train.py:172-174) + add_densification_stats for radii > 0."""
        from . import _C

        empty = dL_dmeans2D.new_empty(0)
        _C.densification_stats(dL_dmeans2D.contiguous(), empty if normal_grad is None else normal_grad.contiguous(),
                               radii.to(dtype=__import__("torch").int32).contiguous(),
                               self.xyz_gradient_accum, self.normal_gradient_accum, self.denom, self.max_radii2D)

    def _reduce_stats(self):
        import torch.distributed as dist

        if self.dist.world > 1:
            for t in (self.xyz_gradient_accum, self.normal_gradient_accum, self.denom):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.dist.group)
            dist.all_reduce(self.max_radii2D, op=dist.ReduceOp.MAX, group=self.dist.group)

    def _full_state(self):
        """Adam states of the whole flat buffer (all-gathered shards when sharded)."""
        import torch
        import torch.distributed as dist

        s = self.shard_size()
        if self.dist.world == 1:
            return self.exp_avg[:self.total()], self.exp_avg_sq[:self.total()]
        out = []
        for t in (self.exp_avg, self.exp_avg_sq):
            full = torch.empty(s * self.dist.world, device=t.device)
            dist.all_gather_into_tensor(full, t.contiguous(), group=self.dist.group)
            out.append(full[:self.total()])
        return out[0], out[1]

    def _densify(self, max_grad, min_opacity, extent, max_screen_size, max_grad_normal, prune_only, noise=None):
        import torch
        import torch.distributed as dist

        from . import _C

        self._reduce_stats()
        m, v = self._full_state()
        flat = self.param[:self.total()]
        counts = [0, 0, 0, 0]
        if self.dist.rank == 0:
            empty = flat.new_empty(0)
            newp, newm, newv, src, Pn, counts = _C.densify_and_prune(
                self.P, self.widths(), self.roles(), flat.contiguous(), m.contiguous(), v.contiguous(),
                self.xyz_gradient_accum, self.normal_gradient_accum, self.denom,
                self.max_radii2D if prune_only else empty, float(max_grad), float(max_grad_normal),
                float(self.percent_dense), float(extent), float(min_opacity), float(max_screen_size or 0.0), 2,
                bool(prune_only), empty if noise is None else noise)
        if self.dist.world > 1:
            hdr = torch.tensor([Pn if self.dist.rank == 0 else 0] + list(counts), device=flat.device)
            dist.broadcast(hdr, 0, group=self.dist.group)
            Pn, counts = int(hdr[0]), [int(x) for x in hdr[1:]]
            if self.dist.rank != 0:
                n = Pn * sum(self.widths())
                newp, newm, newv = (torch.empty(n, device=flat.device) for _ in range(3))
            for t in (newp, newm, newv):
                dist.broadcast(t, 0, group=self.dist.group)
        self.P = int(Pn)
        s = self.shard_size()
        lo, hi = self.shard_range()
        ms, vs = (torch.zeros(s, device=flat.device) for _ in range(2))
        ms[:hi - lo] = newm[lo:hi]
        vs[:hi - lo] = newv[lo:hi]
        self._set_flat(newp, ms, vs)
        if not prune_only:
            self._reset_stats()  # densification_postfix (gaussian_model.py:912-915)
        else:
            # prune_points slices the statistics of the survivors (gaussian_model.py:834-837)
            if self.dist.world > 1:
                if self.dist.rank != 0:
                    src = torch.empty(self.P, dtype=torch.int32, device=flat.device)
                dist.broadcast(src, 0, group=self.dist.group)
            idx = src.long()
            self.xyz_gradient_accum = self.xyz_gradient_accum[idx]
            self.normal_gradient_accum = self.normal_gradient_accum[idx]
            self.denom = self.denom[idx]
            self.max_radii2D = self.max_radii2D[idx]
        return counts

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, max_grad_normal, noise=None):
        """gaussian_model.py:1025-1043. Returns [originals kept, clones kept, split, children kept/k]."""
        return self._densify(max_grad, min_opacity, extent, max_screen_size, max_grad_normal, False, noise)

    def prune(self, min_opacity, extent, max_screen_size):
        """gaussian_model.py:1045-1053."""
        return self._densify(0.0, min_opacity, extent, max_screen_size, 0.0, True)

    def reset_opacity(self):
        """gaussian_model.py:688-691 (the opacity group's Adam state zeroed)."""
        from . import _C

        empty = self.param.new_empty(0)
        _C.reset_opacity(self.P, self.widths(), self.roles(), self.param, empty, empty)
        # zero the opacity state inside this rank's shard
        o = 0
        for n, s in self.groups:
            w = int(np.prod(s))
            if n == "opacity":
                lo, hi = self.shard_range()
                a, b = max(o, lo), min(o + self.P * w, hi)
                if a < b:
                    self.exp_avg[a - lo:b - lo] = 0
                    self.exp_avg_sq[a - lo:b - lo] = 0
            o += self.P * w
