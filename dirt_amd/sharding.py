"""Frame-sharded batched rasterisation across the GPUs of one node (one process per GPU).

The reference has no multi-GPU data path: tests/multi_gpu_test.py:20-29 places two independent renders
on /gpu:0 and /gpu:1 of one session, and GlDispatcher keeps one GL thread per CUDA context
(csrc/gl_dispatcher.h:101-108).  Frames of a batch are independent in both forward and backward
(SURVEY 8e), so the MI355X design shards the batch dimension contiguously over ranks and runs each
shard with no collective in the data path.  The only optional exchange is gathering the rendered
frames (RCCL all-gather over xGMI with the "nccl" backend; gloo works for CPU tensors in tests).
"""
import torch
import torch.distributed as dist

from .rasterise_ops import rasterise_batch


def shard_bounds(batch, rank, world):
    """Contiguous [lo, hi) frame range of `rank`; the first batch % world ranks take one extra frame."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world: %r/%r" % (rank, world))
    base, extra = divmod(int(batch), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _wire(local, dtype):
    """The block as it travels: `local` itself, or cast to the reduced-precision `dtype` (torch.bfloat16 /
    torch.float16: half the xGMI bytes of float32 pixels; the gathered batch keeps that dtype)."""
    if dtype is None or dtype == local.dtype:
        return local
    if dtype not in (torch.bfloat16, torch.float16):
        raise ValueError("gather dtype must be None, torch.bfloat16 or torch.float16, got %r" % (dtype,))
    return local.to(dtype)


def gather_frames(local, batch, group=None, dtype=None):
    """All-gather per-rank frame blocks [b_r, ...] into the full batch [batch, ...] on every rank.

    Pads every block to the largest shard so one all_gather (RCCL ring over xGMI) moves it.  dtype:
    optional reduced-precision wire format (see _wire)."""
    local = _wire(local, dtype)
    world = dist.get_world_size(group)
    sizes = [shard_bounds(batch, r, world) for r in range(world)]
    mx = max(hi - lo for lo, hi in sizes)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[: hi - lo] for o, (lo, hi) in zip(outs, sizes)], 0)


def gather_frames_to(local, batch, dst=0, group=None, dtype=None):
    """Gather per-rank frame blocks into the full batch on rank `dst` only ("ncclGather to rank 0 if
    only one consumer"); returns the batch on `dst` and None on the other ranks.  Every rank sends its block
    once (RCCL send / recv over xGMI with the "nccl" backend); the root's ingress bounds it like the
    all-gather's per-rank ingress, but the other ranks receive nothing.  dtype: optional
    reduced-precision wire format (see _wire)."""
    work, finish = gather_frames_to_async(local, batch, dst=dst, group=group, dtype=dtype)
    return finish()


def gather_frames_to_async(local, batch, dst=0, group=None, dtype=None):
    """gather_frames_to started asynchronously: returns (work, finish); finish() -> the batch on `dst`, None
    elsewhere.  For a pipelined single consumer: the next step renders while this step's frames move to the
    root."""
    local = _wire(local, dtype)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [shard_bounds(batch, r, world) for r in range(world)]
    mx = max(hi - lo for lo, hi in sizes)
    if local.shape[0] == mx:
        pad = local.contiguous()
    else:
        pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    via_host = pad.is_cuda and dist.get_backend(group) == "gloo"  # gloo moves host memory only
    src = pad.cpu() if via_host else pad
    outs = [torch.empty_like(src) for _ in range(world)] if rank == dst else None
    work = dist.gather(src, gather_list=outs, dst=dst, group=group, async_op=True)

    def finish():
        work.wait()
        if rank != dst:
            return None
        full = torch.cat([o[: hi - lo] for o, (lo, hi) in zip(outs, sizes)], 0)
        return full.to(local.device) if via_host else full

    return work, finish


def gather_frames_async(local, batch, group=None, dtype=None):
    """Start gathering per-rank frame blocks; returns (work, finish) where finish() -> the full batch.

    The collective runs on the backend's own stream (RCCL: its NCCL stream, which waits for the work
    already queued on the current stream), so the caller can queue the next step's render while the
    frames move over xGMI; work.wait() makes the current stream wait for the gather.  dtype: optional
    reduced-precision wire format (see _wire; the cast is queued on the current stream)."""
    local = _wire(local, dtype)
    world = dist.get_world_size(group)
    sizes = [shard_bounds(batch, r, world) for r in range(world)]
    mx = max(hi - lo for lo, hi in sizes)
    if local.shape[0] == mx:
        pad = local.contiguous()
    else:
        pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    via_host = pad.is_cuda and dist.get_backend(group) == "gloo"  # gloo moves host memory only
    src = pad.cpu() if via_host else pad
    out = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=src.device)
    work = dist.all_gather_into_tensor(out, src, group=group, async_op=True)

    def finish():
        nonlocal out
        work.wait()
        if via_host:
            out = out.to(local.device)
        if all(hi - lo == mx for lo, hi in sizes):
            return out
        return torch.cat([out[r * mx: r * mx + hi - lo] for r, (lo, hi) in enumerate(sizes)], 0)

    return work, finish


class _SharedGradAllReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, grad):
        grad = grad.contiguous().clone()
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=ctx.group)
        return grad, None


def shared_across_ranks(x, group=None):
    """Mark a tensor that every rank's frames use (e.g. one mesh's vertices tiled over the batch,
    tests/rasterise_tests.py:89): identity forward; in the backward its gradient is summed over the ranks
    (one all-reduce: RCCL over xGMI with the "nccl" backend), so every rank ends up with the
    gradient of the whole batch, as if one process had rendered every frame.  ~16 V bytes per step."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    return _SharedGradAllReduce.apply(x, group)


def allreduce_shared_gradient(grad, group=None, async_op=False):
    """The collective of a data-parallel fit of one shared mesh (tests/rasterise_tests.py:89 tiles one mesh
    over the batch): this rank's per-frame gradient `grad` [b_local, ...] (e.g. RasteriseSession's
    grad_vertices) is summed over its frames, then over the ranks with one all-reduce (RCCL over xGMI with the
    "nccl" backend).  Returns the batch's gradient [...] on every rank (and the work handle if async_op).
    The same sum shared_across_ranks produces inside autograd, for callers that drive the op without it."""
    total = grad.sum(0) if grad.dim() > 0 and grad.shape[0] != 1 else grad.reshape(grad.shape[1:]).clone()
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return (total, None) if async_op else total
    work = dist.all_reduce(total, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    return (total, work) if async_op else total


def rasterise_batch_sharded(background, vertices, vertex_colors, faces, camera_pos=None, height=None, width=None,
                            channels=None, group=None, gather=False, render=rasterise_batch, gather_dtype=None):
    """rasterise_batch over this rank's contiguous share of the frames.

    Every rank passes the full batch (or any object supporting slicing on dim 0); the rank renders
    frames [lo, hi) and returns (pixels_local, (lo, hi)), or the gathered full batch if `gather`.
    Gradients flow through pixels_local like rasterise_batch; the gathered tensor is forward-only.
    `render` is the per-shard renderer (the HIP op by default); `gather_dtype` the optional reduced-precision
    wire format of the gather (torch.bfloat16 / torch.float16)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    B = background.shape[0]
    lo, hi = shard_bounds(B, rank, world)
    local = render(background[lo:hi], vertices[lo:hi], vertex_colors[lo:hi], faces[lo:hi], camera_pos=camera_pos,
                   height=height, width=width, channels=channels)
    if not gather:
        return local, (lo, hi)
    if world == 1:
        return _wire(local.detach(), gather_dtype)
    with torch.no_grad():
        return gather_frames(local.detach(), B, group=group, dtype=gather_dtype)
