"""Multi-process (world_size 2, gloo, CPU) tests of the frame-sharded batch path (dirt_amd.sharding).

The HIP renderer needs a GPU, so the per-shard renderer here is the CPU oracle; what is under test is
the partition, the no-collective local path and the all-gather of the rendered frames
(reference multi-device check: tests/multi_gpu_test.py:6-29, SURVEY 8c 'Multi-device').
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import scenes
from dirt_amd.sharding import (allreduce_shared_gradient, gather_frames, gather_frames_async, gather_frames_to,
                               gather_frames_to_async, rasterise_batch_sharded, shard_bounds, shared_across_ranks)
from oracle import oracle


def test_shard_bounds_partition():
    for B in (0, 1, 5, 8, 64, 65):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _oracle_render(bg, v, c, f, camera_pos=None, height=None, width=None, channels=None):
    px, _, _ = oracle.rasterise_fwd(bg.numpy(), v.numpy(), c.numpy(), f.numpy())
    return torch.from_numpy(px)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, inputs, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bg, v, c, f = (torch.from_numpy(a) for a in inputs)
        local, (lo, hi) = rasterise_batch_sharded(bg, v, c, f, render=_oracle_render)
        full = gather_frames(local, bg.shape[0])
        full2 = rasterise_batch_sharded(bg, v, c, f, render=_oracle_render, gather=True)
        work, finish = gather_frames_async(local, bg.shape[0])
        full3 = finish()
        root = gather_frames_to(local, bg.shape[0], dst=1)  # the single-consumer gather: rank 1 only
        root = None if root is None else root.numpy()
        # reduced-precision wire formats (half the xGMI bytes): every path returns the cast batch
        red = {}
        for dt in (torch.bfloat16, torch.float16):
            a = gather_frames(local, bg.shape[0], dtype=dt)
            b = gather_frames_async(local, bg.shape[0], dtype=dt)[1]()
            r0 = gather_frames_to_async(local, bg.shape[0], dst=0, dtype=dt)[1]()
            g2 = rasterise_batch_sharded(bg, v, c, f, render=_oracle_render, gather=True, gather_dtype=dt)
            assert a.dtype == b.dtype == g2.dtype == dt and (r0 is None) == (rank != 0)
            red[str(dt)] = (a.float().numpy(), b.float().numpy(), None if r0 is None else r0.float().numpy(),
                            g2.float().numpy())
        # a parameter shared by every rank's frames: its gradient is summed over the ranks
        x = torch.arange(6, dtype=torch.float32).requires_grad_(True)
        loss = (shared_across_ranks(x) * (rank + 1)).sum() + (x * x).sum() * 0.0
        loss.backward()
        # bench.py's legs.shared_allreduce collective: per-frame gradients of this rank's frames, summed over
        # the frames and then the ranks (frame k's gradient is k + 1 everywhere, so the batch sum is known)
        per_frame = torch.stack([torch.full((7, 4), float(k + 1)) for k in range(lo, hi)]) if hi > lo else \
            torch.zeros((0, 7, 4))
        total = allreduce_shared_gradient(per_frame) if hi - lo != 0 else None
        t2, work = allreduce_shared_gradient(per_frame, async_op=True) if hi - lo != 0 else (None, None)
        if work is not None:
            work.wait()
        red["allreduce"] = (None if total is None else total.numpy(), None if t2 is None else t2.numpy())
        outq.put((rank, lo, hi, local.numpy(), full.numpy(), full2.numpy(), full3.numpy(), x.grad.numpy(), root, red))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [5, 4])
def test_two_rank_sharded_batch_matches_single_process(B):
    inputs = scenes.batch_of(scenes.random_triangles, B, F=150, W=40, H=32, radius_px=8.0, seed=3)
    ref, _, _ = oracle.rasterise_fwd(*inputs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, inputs, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    covered = []
    for rank, lo, hi, local, full, full2, full3, xgrad, root, red in res:
        want_sum = np.full((7, 4), B * (B + 1) / 2, np.float32)  # sum over the batch's frames of (k + 1)
        for got in red["allreduce"]:
            np.testing.assert_array_equal(got, want_sum)
        for dt in (torch.bfloat16, torch.float16):
            want = torch.from_numpy(ref).to(dt).float().numpy()
            for k, got in enumerate(red[str(dt)]):
                if got is not None:
                    np.testing.assert_array_equal(got, want)
        assert red[str(torch.bfloat16)][2] is not None if rank == 0 else red[str(torch.bfloat16)][2] is None
        np.testing.assert_array_equal(full3, ref)          # the async all_gather_into_tensor path
        if rank == 1:
            np.testing.assert_array_equal(root, ref)       # gather to one root reassembles the batch there
        else:
            assert root is None
        np.testing.assert_array_equal(xgrad, np.full(6, 3.0, np.float32))  # (1 + 2) summed over ranks
        assert (lo, hi) == shard_bounds(B, rank, 2)
        np.testing.assert_array_equal(local, ref[lo:hi])   # each rank renders only its frames
        np.testing.assert_array_equal(full, ref)           # all-gather reassembles the batch
        np.testing.assert_array_equal(full2, ref)
        covered.extend(range(lo, hi))
    assert covered == list(range(B))
