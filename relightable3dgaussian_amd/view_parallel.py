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

The SH block is 48 of those 70 floats, yet one view's SH gradient is rank 1 per Gaussian:
dL/dsh[k][c] = Y_k(dir_v) * dRGB_v[c] (backward.cu:20-139), with dir_v = normalize(mean -
campos_v) known to every rank. So the default exchange ("views") all-reduces only the other 22
floats and ALL-GATHERS each view's clamp-masked colour gradient dRGB (3 floats per Gaussian);
every rank then rebuilds sum_v Y(dir_v) dRGB_v on the device (r3dg_sh_grad_from_views). Per GPU
on an N-rank ring that moves 2 (N-1)/N * 88 + (N-1) * 12 bytes per Gaussian instead of
2 (N-1)/N * 280: 238 vs 490 B at N = 8 (2.06x fewer link bytes), and the rebuilt sum is
identical on every rank (fixed view order).
"""
from __future__ import annotations

import math

import numpy as np

# index into the `_C.rasterize_gaussians_backward` result tuple
# (means2D, colors, opacity, means3D, features, cov3D, sh, scales, rotations)
GRAD_FIELDS = (("means3D", 3), ("sh", 6), ("opacity", 2), ("scales", 7), ("rotations", 8), ("features", 4))


SH_INDEX = 6
COLOR_INDEX = 1
# the fields still all-reduced when the SH block travels as per-view colour gradients
DENSE_FIELDS = tuple(f for f in GRAD_FIELDS if f[0] != "sh")


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


def gather_campos(campos, group=None):
    """[N, 3]: every rank's camera centre, in rank order."""
    import torch
    import torch.distributed as dist

    c = campos.reshape(1, 3).contiguous()
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return c
    parts = [torch.empty_like(c) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, c, group=group)
    return torch.cat(parts)


def exchange_grads_views(grads, drgb, campos, means3D, degree, rebuild, group=None) -> dict:
    """The "views" exchange, unchunked: all-reduce the dense fields, all-gather this view's
    clamp-masked colour gradients drgb [P,3] and camera centre, and rebuild the SH gradient sum
    with rebuild(means3D, campos [N,3], drgb [N,P,3], degree, M) -> [P,M,3] (the device kernel
    r3dg_sh_grad_from_views; tests pass the CPU oracle). Returns name -> summed tensor."""
    import torch
    import torch.distributed as dist

    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    flat = torch.cat([grads[i].reshape(-1) for _, i in DENSE_FIELDS])
    if multi:
        dist.all_reduce(flat, group=group)
    out, o = {}, 0
    for name, i in DENSE_FIELDS:
        n = grads[i].numel()
        out[name] = flat[o:o + n].view_as(grads[i])
        o += n
    cams = gather_campos(campos, group)
    d = drgb.contiguous()
    if multi:
        parts = [torch.empty_like(d) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, d, group=group)
        d_all = torch.stack(parts)
    else:
        d_all = d[None]
    out["sh"] = rebuild(means3D, cams, d_all, degree, grads[SH_INDEX].shape[1])
    return out


_COMM = {}


def _all_gather_into(buf, d, group=None):
    """Async all-gather of d into buf [N, ...] (one contiguous output on RCCL; per-rank views on
    other backends)."""
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return dist.all_gather_into_tensor(buf, d, group=group, async_op=True)
    return dist.all_gather(list(buf.unbind(0)), d, group=group, async_op=True)


# index of the packed [P, 11 + S] dense-gradient array in the chunk callback's outputs
# (_C.rasterize_gaussians_backward_chunked_packed: means3D 3 | opacity 1 | scales 3 | rotations 4 |
# features S per row, the DENSE_FIELDS in order)
PACKED_INDEX = 9
# collectives issued by the last backward_all_reduce call (bench.py reports it per step)
LAST_COLLECTIVES = {"count": 0, "sequence": []}


def _comm_stream(stream=None):
    import torch

    if stream is not None:
        return stream
    cur = torch.cuda.current_stream()
    return _COMM.setdefault(cur.device, torch.cuda.Stream(device=cur.device))


def _after_current(comm):
    """The communication stream waits for what the compute stream has enqueued so far."""
    import torch

    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    comm.wait_event(ev)


def chunk_all_reduce_hook(works: list, seq: list, group=None, stream=None):
    """Chunk callback for `_C.rasterize_gaussians_backward_chunked_packed`: all-reduces the chunk's
    rows of the packed dense array (one contiguous span) and of the SH block on a communication
    stream that first waits for the chunk's kernels, while the compute stream goes on with the next
    chunk. `works` collects the async handles, `seq` the (kind, floats) of each collective."""
    import torch
    import torch.distributed as dist

    def hook(chunk, g0, g1, outs):
        comm = _comm_stream(stream)
        _after_current(comm)
        with torch.cuda.stream(comm):
            for t in (outs[PACKED_INDEX], outs[SH_INDEX]):
                if t.numel():
                    works.append(dist.all_reduce(t[g0:g1], group=group, async_op=True))
                    seq.append(("all_reduce", t[g0:g1].numel()))

    return hook


def chunk_views_hook(_C, works: list, gathered: list, seq: list, geom, P: int, group=None, stream=None):
    """Chunk callback of the "views" exchange: the chunk's rows of the packed dense array (22
    floats per Gaussian at S = 11, one contiguous span) are all-reduced and its clamp-masked colour
    gradients (r3dg_sh_color_grads, enqueued on the compute stream behind the chunk's kernels)
    all-gathered into [N, n, 3], both on the communication stream: two collectives per chunk."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)

    def hook(chunk, g0, g1, outs):
        sh_on = outs[SH_INDEX].numel() > 0
        d = _C.sh_color_grads(geom, P, outs[COLOR_INDEX], g0, g1) if sh_on else None
        comm = _comm_stream(stream)
        _after_current(comm)
        with torch.cuda.stream(comm):
            dense = outs[PACKED_INDEX][g0:g1]
            works.append(dist.all_reduce(dense, group=group, async_op=True))
            seq.append(("all_reduce", dense.numel()))
            if sh_on:
                buf = torch.empty((world, g1 - g0, 3), dtype=d.dtype, device=d.device)
                works.append(_all_gather_into(buf, d, group))
                seq.append(("all_gather", d.numel()))
                gathered.append((g0, buf, d, len(works)))  # the chunk's exchange = works[:len]

    return hook


def gather_campos_async(campos, group=None, stream=None):
    """Start the all-gather of every rank's camera centre ([N, 3], rank order) on the
    communication stream; returns (buffer, work) -- wait on the work before reading the buffer."""
    import torch
    import torch.distributed as dist

    comm = _comm_stream(stream)
    _after_current(comm)
    c = campos.reshape(1, 3).contiguous()
    with torch.cuda.stream(comm):
        buf = torch.empty((dist.get_world_size(group), 1, 3), dtype=c.dtype, device=c.device)
        work = _all_gather_into(buf, c, group)
    return buf, work


def backward_all_reduce(_C, bwd_args, n_chunks: int = 4, group=None, sh_exchange: str = "views"):
    """rasterize_gaussians_backward_chunked_packed(*bwd_args, n_chunks, hook) with the per-Gaussian
    gradients summed over ranks chunk by chunk, overlapped with the remaining per-Gaussian kernels
    (the blend must finish before any Gaussian's gradient is final, so only that phase overlaps).
    `bwd_args` is the rasterize_gaussians_backward_ex argument list + (color_hwc, feature_native).
    sh_exchange "views" (default) all-gathers per-view colour gradients and rebuilds the SH sum
    on every rank; "allreduce" all-reduces the SH block like the other fields. Per step: one
    asynchronous all-gather of the camera centres ("views") + two collectives per chunk (9 at 4
    chunks; LAST_COLLECTIVES records them). Returns the backward 9-tuple (the dense gradients are
    column views of one packed array); the current stream waits for the exchange."""
    import torch
    import torch.distributed as dist

    works, gathered, seq = [], [], []
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    if not multi:
        LAST_COLLECTIVES.update(count=0, sequence=[])
        return _C.rasterize_gaussians_backward_chunked(*bwd_args, 1, None)
    if sh_exchange == "allreduce":
        hook = chunk_all_reduce_hook(works, seq, group)
    else:
        means3D, sh, degree, campos, geom = bwd_args[1], bwd_args[17], bwd_args[18], bwd_args[19], bwd_args[20]
        cams_buf, cams_work = gather_campos_async(campos, group)
        seq.append(("all_gather", 3))
        hook = chunk_views_hook(_C, works, gathered, seq, geom, means3D.shape[0], group)
    grads = _C.rasterize_gaussians_backward_chunked_packed(*bwd_args, n_chunks, hook)
    cur = torch.cuda.current_stream()
    done = 0
    if gathered:
        cams_work.wait()
        cams = cams_buf.reshape(-1, 3)
        cams_buf.record_stream(cur)
    for g0, buf, _, upto in gathered:
        # every rank rebuilds the same SH gradient sum, chunk by chunk: a chunk's rebuild waits for
        # that chunk's collectives only and overlaps the later chunks' communication
        for w in works[done:upto]:
            w.wait()
        done = upto
        _C.sh_grad_from_views(means3D, cams, buf, degree, g0, grads[SH_INDEX])
        buf.record_stream(cur)  # allocated on the communication stream, read here
    for w in works[done:]:
        w.wait()
    if sh_exchange != "allreduce" and not gathered:
        cams_work.wait()
    LAST_COLLECTIVES.update(count=len(seq), sequence=seq)
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
