"""View-parallel data parallelism around the rasterizer.

The reference trains one camera per iteration on one GPU (train.py: render -> loss -> backward ->
optimizer step). Here every rank renders its own camera of the SAME replicated Gaussian set and
the per-Gaussian gradients are summed across ranks with one collective per step -- the gradient of
the multi-view loss sum_r L_r, i.e. what the reference would get by accumulating `world` views.
The rasterizer itself has no exchange step (tiles of a view are independent), so the only
collective is this all-reduce of one flat bucket:

    means3D 3 + sh 3*M + opacity 1 + scales 3 + rotations 4 + features S    floats per Gaussian

(70 at M=16, S=11; 280 MB for 1M Gaussians -- one bucket, which on xGMI ring all-reduce is
link-bandwidth bound, so it is issued once per step rather than per tensor).
"""
from __future__ import annotations

import math

import numpy as np

# index into the `_C.rasterize_gaussians_backward` result tuple
# (means2D, colors, opacity, means3D, features, cov3D, sh, scales, rotations)
GRAD_FIELDS = (("means3D", 3), ("sh", 6), ("opacity", 2), ("scales", 7), ("rotations", 8), ("features", 4))


def flatten_grads(grads):
    """Concatenate the exchanged gradients of a backward tuple into one flat bucket."""
    import torch

    return torch.cat([grads[i].reshape(-1) for _, i in GRAD_FIELDS])


def unflatten_grads(flat, grads) -> dict:
    """Split a flat bucket back into tensors shaped like `grads` (dict name -> tensor view)."""
    out, o = {}, 0
    for name, i in GRAD_FIELDS:
        n = grads[i].numel()
        out[name] = flat[o:o + n].view_as(grads[i])
        o += n
    return out


def all_reduce_grads(grads, group=None) -> dict:
    """Sum the per-Gaussian gradients of every rank's view (one all-reduce, RCCL on GPU, gloo on
    CPU). Returns name -> summed tensor."""
    import torch.distributed as dist

    flat = flatten_grads(grads)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat, group=group)
    return unflatten_grads(flat, grads)


_COMM = {}


def chunk_all_reduce_hook(works: list, group=None, stream=None):
    """Chunk callback for `_C.rasterize_gaussians_backward_chunked`: all-reduces the exchanged
    gradient slices of Gaussians [g0, g1) (rows of contiguous [P, ...] tensors, so each slice is
    contiguous) on a communication stream that first waits for the chunk's kernels, while the
    compute stream goes on with the next chunk. `works` collects the async handles."""
    import torch
    import torch.distributed as dist

    def hook(chunk, g0, g1, outs):
        cur = torch.cuda.current_stream()
        comm = stream
        if comm is None:
            comm = _COMM.setdefault(cur.device, torch.cuda.Stream(device=cur.device))
        ev = torch.cuda.Event()
        ev.record(cur)
        comm.wait_event(ev)
        with torch.cuda.stream(comm):
            for _, i in GRAD_FIELDS:
                t = outs[i]
                if t.numel():
                    works.append(dist.all_reduce(t[g0:g1], group=group, async_op=True))

    return hook


def backward_all_reduce(_C, bwd_args, n_chunks: int = 4, group=None):
    """rasterize_gaussians_backward_chunked(*bwd_args, n_chunks, hook) with the exchanged fields
    summed over ranks chunk by chunk, overlapped with the remaining per-Gaussian kernels (the
    blend must finish before any Gaussian's gradient is final, so only that phase overlaps).
    `bwd_args` is the rasterize_gaussians_backward_ex argument list + (color_hwc, feature_native).
    Returns the backward 9-tuple; the current stream waits for the exchange."""
    import torch.distributed as dist

    works = []
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    hook = chunk_all_reduce_hook(works, group) if multi else None
    grads = _C.rasterize_gaussians_backward_chunked(*bwd_args, n_chunks if multi else 1, hook)
    for w in works:
        w.wait()
    return grads


def rank_yaw(rank: int, world: int, step_deg: float = 1.0) -> np.ndarray:
    """Rotation of rank `rank`'s camera: a small yaw so every view costs about the same."""
    if world == 1:
        return np.eye(3)
    yaw = math.radians((rank - (world - 1) / 2.0) * step_deg)
    return np.array([[math.cos(yaw), 0, math.sin(yaw)], [0, 1, 0], [-math.sin(yaw), 0, math.cos(yaw)]])


def rank_camera(base, rank: int, world: int, step_deg: float = 1.0):
    """`base` (synthetic.Camera at the origin looking down +z) turned by rank_yaw."""
    from . import synthetic

    if world == 1:
        return base
    return synthetic.make_camera(rank_yaw(rank, world, step_deg), np.zeros(3), base.fovx, base.fovy, base.width,
                                 base.height)
