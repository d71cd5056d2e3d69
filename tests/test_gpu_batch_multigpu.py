"""GPU: BASELINE config 5's per-rank shard, the RCCL collectives of dirt_amd.sharding on HBM tensors, and
the public autograd path's workspace handling.

* C5 = 64 frames x 20k triangles x 1024^2 sharded over 8 GPUs: one rank's shard (8 frames) fwd+bwd through
  rasterise_batch, every frame's g-buffer and pixels bit-exact, two frames' gradients in tolerance.
* gather_frames / gather_frames_async / shared_across_ranks with the "nccl" (RCCL) backend at world size 1
  on device tensors (the multi-rank runs are the driver's 8-GPU node; tests/test_sharding.py covers 2 ranks
  over gloo), so RCCL init and its all_gather / all_reduce run on the card.
* autograd path: cached scratch across layouts, forward zero-filled gradient buffers (one backward) and a
  retained graph's second backward, opt-in face-index checks.
"""
import os
import socket

import numpy as np
import pytest
import torch

import scenes
from oracle import oracle
from test_gpu_parity import assert_close_grad, _gpu

pytestmark = pytest.mark.gpu


def test_config5_per_rank_shard_fwd_bwd():
    """C5's per-rank shard (bench.py c5: 8 frames x 20k tris x 1024^2, seeds 0..7) through the public op."""
    import dirt_amd
    frames = [scenes.random_triangles(F=20000, W=1024, H=1024, seed=b) for b in range(8)]
    bg, v, c, f = (np.stack([fr[k] for fr in frames]) for k in range(4))
    gp = np.random.default_rng(10_000).standard_normal(bg.shape).astype(np.float32)
    t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
    px, gbuf = dirt_amd.rasterise_ops._rasterise_batched(t[0], t[1], t[2], _gpu(f), None, 1024, 1024, 3, 0,
                                                         return_gbuffer=True)
    gbg, gv, gc = torch.autograd.grad(px, t, _gpu(gp))
    ref_px, ref_gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    np.testing.assert_array_equal(gbuf.cpu().numpy(), ref_gb)
    np.testing.assert_array_equal(px.detach().cpu().numpy(), ref_px)
    for b in (0, 5):
        rgv, rgc, rgbg = oracle.rasterise_bwd(v[b:b + 1], c[b:b + 1], f[b:b + 1], ref_px[b:b + 1], gp[b:b + 1],
                                              ref_gb[b:b + 1])
        np.testing.assert_array_equal(gbg[b:b + 1].cpu().numpy(), rgbg)
        assert_close_grad(gv[b:b + 1].cpu().numpy(), rgv, "grad_vertices frame %d" % b)
        assert_close_grad(gc[b:b + 1].cpu().numpy(), rgc, "grad_vertex_colors frame %d" % b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _nccl_worker(port, inputs, outq):
    import torch.distributed as dist
    from dirt_amd.sharding import (gather_frames, gather_frames_async, gather_frames_to, gather_frames_to_async,
                                   rasterise_batch_sharded, shared_across_ranks)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        dev = torch.device("cuda", 0)
        bg, v, c, f = (torch.from_numpy(a).to(dev) for a in inputs)
        local, (lo, hi) = rasterise_batch_sharded(bg, v, c, f)
        full = gather_frames(local, bg.shape[0])
        work, finish = gather_frames_async(local, bg.shape[0])
        full2 = finish()
        full3 = rasterise_batch_sharded(bg, v, c, f, gather=True)
        full4 = gather_frames_to(local, bg.shape[0], dst=0)  # RCCL gather to one root
        assert full.is_cuda and full2.is_cuda and full4.is_cuda
        # reduced-precision wire formats over RCCL (half the xGMI bytes) and the async root gather
        red = [gather_frames(local, bg.shape[0], dtype=torch.bfloat16),
               gather_frames_async(local, bg.shape[0], dtype=torch.bfloat16)[1](),
               gather_frames_to_async(local, bg.shape[0], dst=0, dtype=torch.float16)[1](),
               gather_frames_to_async(local, bg.shape[0], dst=0)[1]()]
        assert [t.dtype for t in red] == [torch.bfloat16, torch.bfloat16, torch.float16, torch.float32]
        # a parameter shared by the rank's frames: all_reduce over RCCL (world 1: the identity)
        x = torch.arange(6, dtype=torch.float32, device=dev).requires_grad_(True)
        (shared_across_ranks(x) * 2.0).sum().backward()
        # explicit RCCL all_reduce on the card (shared_across_ranks skips the collective at world size 1)
        y = torch.ones(1000, device=dev)
        dist.all_reduce(y)
        torch.cuda.synchronize()
        outq.put((lo, hi, full.cpu().numpy(), full2.cpu().numpy(), full3.cpu().numpy(), full4.cpu().numpy(),
                  x.grad.cpu().numpy(), float(y.sum()), [t.float().cpu().numpy() for t in red]))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_gather_and_allreduce_on_device():
    import torch.multiprocessing as mp
    inputs = scenes.batch_of(scenes.random_triangles, 3, F=400, W=64, H=48, radius_px=8.0, seed=70)
    ref, _, _ = oracle.rasterise_fwd(*inputs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), inputs, q))
    p.start()
    res = None
    for _ in range(120):  # poll, so that a worker that dies fails the test instead of hanging it
        try:
            res = q.get(timeout=1)
            break
        except Exception:
            if not p.is_alive():
                break
    assert res is not None, "nccl worker exited with %s" % p.exitcode
    lo, hi, full, full2, full3, full4, xgrad, ysum, red = res
    p.join(timeout=120)
    assert p.exitcode == 0
    assert (lo, hi) == (0, 3)
    for a in (full, full2, full3, full4, red[3]):
        np.testing.assert_array_equal(a, ref)
    rt = torch.from_numpy(ref)
    np.testing.assert_array_equal(red[0], rt.bfloat16().float().numpy())
    np.testing.assert_array_equal(red[1], rt.bfloat16().float().numpy())
    np.testing.assert_array_equal(red[2], rt.half().float().numpy())
    np.testing.assert_array_equal(xgrad, np.full(6, 2.0, np.float32))
    assert ysum == 1000.0


def test_autograd_workspace_cache_and_retained_graph():
    """Repeated calls reuse one cached scratch per layout (it stays clean across forwards); a retained
    graph's second backward gives the same gradients as the first (the forward's zero-filled buffers
    serve only the first)."""
    import dirt_amd
    from dirt_amd import rasterise_ops
    rasterise_ops.workspace_cache_clear()
    scs = [scenes.random_triangles(F=900, W=96, H=80, radius_px=10.0, seed=s) for s in (81, 82)]
    scs.append(scenes.random_triangles(F=500, W=64, H=48, radius_px=8.0, seed=83))
    for rep in range(3):
        for bg, v, c, f in scs:
            t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
            px = dirt_amd.rasterise(t[0], t[1], t[2], _gpu(f))
            ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
            np.testing.assert_array_equal(px.detach().cpu().numpy(), ref[0])
    assert rasterise_ops.workspace_cache_size() == 2  # two layouts (F, H, W differ), one stream
    bg, v, c, f = scs[0]
    t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
    px = dirt_amd.rasterise(t[0], t[1], t[2], _gpu(f))
    g = torch.randn_like(px)
    first = [x.clone() for x in torch.autograd.grad(px, t, g, retain_graph=True)]
    second = torch.autograd.grad(px, t, g)
    for a, b in zip(first, second):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(a.abs().max()))
    # .backward() accumulation into .grad over two forwards
    for x in t:
        x.grad = None
    for _ in range(2):
        dirt_amd.rasterise(t[0], t[1], t[2], _gpu(f)).backward(g)
    for a, x in zip(first, t):
        torch.testing.assert_close(x.grad, 2 * a, rtol=1e-5, atol=1e-5 * float(a.abs().max()))


def test_autograd_matches_session():
    import dirt_amd
    from dirt_amd.session import RasteriseSession
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=3000, W=256, H=192, radius_px=12.0, seed=84))
    ts = [_gpu(a) for a in (bg, v, c, f)]
    g = torch.randn(bg.shape, device="cuda")
    sess = RasteriseSession(*bg.shape, v.shape[1], f.shape[1], device="cuda")
    sess.forward(*ts)
    sgb, sgv, sgc = sess.backward(g)
    t = [x.clone().requires_grad_(True) for x in ts[:3]]
    px = dirt_amd.rasterise_batch(t[0], t[1], t[2], ts[3])
    agb, agv, agc = torch.autograd.grad(px, t, g)
    assert torch.equal(px, sess.pixels)
    assert torch.equal(agb, sgb)
    torch.testing.assert_close(agv, sgv, rtol=1e-5, atol=1e-5 * float(sgv.abs().max()))
    torch.testing.assert_close(agc, sgc, rtol=1e-5, atol=1e-5 * float(sgc.abs().max()))


def test_check_faces_opt_in():
    import dirt_amd
    bg, v, c, f = scenes.random_triangles(F=50, W=32, H=32, seed=9)
    bad = f.copy()
    bad[7] = [0, 1, 10 ** 6]
    # default: no check, the face is culled (oracle agrees)
    px = dirt_amd.rasterise(_gpu(bg), _gpu(v), _gpu(c), _gpu(bad))
    ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], bad[None])
    np.testing.assert_array_equal(px.cpu().numpy(), ref[0])
    with pytest.raises(IndexError, match="out of range"):
        dirt_amd.rasterise(_gpu(bg), _gpu(v), _gpu(c), _gpu(bad), check_faces=True)
    bad[7] = [-1, 1, 2]
    with pytest.raises(IndexError):
        dirt_amd.rasterise_batch(_gpu(bg[None]), _gpu(v[None]), _gpu(c[None]), _gpu(bad[None]), check_faces=True)
    ok = dirt_amd.rasterise(_gpu(bg), _gpu(v), _gpu(c), _gpu(f), check_faces=True)
    ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
    np.testing.assert_array_equal(ok.cpu().numpy(), ref[0])


def test_hip_graph_capture_of_autograd_path():
    """The public op + autograd captured into one HIP graph (cached scratch warmed on the capture stream)
    and replayed: results equal the eager call."""
    import dirt_amd
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=2000, W=160, H=128, radius_px=10.0, seed=85))
    t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
    ft = _gpu(f)
    g = torch.randn(bg.shape, device="cuda")
    outs = {}

    def step():
        px = dirt_amd.rasterise_batch(t[0], t[1], t[2], ft)
        outs["px"] = px
        outs["grads"] = torch.autograd.grad(px, t, g)

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        step()
    torch.cuda.synchronize()
    ref_px = outs["px"].detach().clone()
    ref_g = [x.clone() for x in outs["grads"]]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        step()
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(outs["px"], ref_px)
    assert torch.equal(outs["grads"][0], ref_g[0])
    for a, b in zip(outs["grads"][1:], ref_g[1:]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()))


@pytest.mark.parametrize("impl", ["ext", "py"])
def test_captured_graph_survives_cache_eviction_and_clear(impl):
    """a HIP graph captured through the public op replays writes into the op's scratch.  After
    capture, clearing the cache and churning it with other layouts must not free that scratch (since round 5
    it lives in the graph's own memory pool).  Capture, clear + evict + allocate over the freed pool, replay,
    compare with the eager result."""
    from dirt_amd import rasterise_ops
    ext = rasterise_ops._torch_ext()
    if impl == "ext":
        assert ext is not None

    def op(t0, t1, t2, ft, H, W, C):
        args = (t0, t1, t2, ft, None, H, W, C, 0, 0, False, False)
        return ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args)

    rasterise_ops.workspace_cache_clear(force=True)
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=86))
    B, H, W, C = bg.shape
    t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
    ft = _gpu(f)
    g = torch.randn(bg.shape, device="cuda")
    outs = {}

    def step():
        px, _ = op(t[0], t[1], t[2], ft, H, W, C)
        outs["px"] = px
        outs["grads"] = torch.autograd.grad(px, t, g)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.synchronize()
    ref_px = outs["px"].detach().clone()
    ref_g = [x.clone() for x in outs["grads"]]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        step()
    torch.cuda.synchronize()
    # churn the cache: clear (non-forced) and six other layouts on the default stream, then fill fresh
    # allocations with garbage so that a freed scratch would be overwritten
    rasterise_ops.workspace_cache_clear()
    for k in range(6):
        bg2, v2, c2, f2 = (a[None] for a in scenes.random_triangles(F=300 + 50 * k, W=48 + 8 * k, H=40, seed=87 + k))
        op(_gpu(bg2), _gpu(v2), _gpu(c2), _gpu(f2), 40, 48 + 8 * k, 3)
    junk = [torch.full((1 << 22,), -7, dtype=torch.int32, device="cuda") for _ in range(16)]
    torch.cuda.synchronize()
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(outs["px"], ref_px)
    assert torch.equal(outs["grads"][0], ref_g[0])
    for a, b in zip(outs["grads"][1:], ref_g[1:]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()))
    del junk, graph
    rasterise_ops.workspace_cache_clear(force=True)
    assert rasterise_ops.workspace_cache_size() == 0


@pytest.mark.filterwarnings("error:The AccumulateGrad node's stream does not match")
@pytest.mark.parametrize("shared_pool", [False, True])
@pytest.mark.parametrize("impl", ["ext", "py"])
def test_two_graphs_same_layout_second_replayed_first(impl, shared_pool):
    """two graphs captured through the public op with the same layout (torch.cuda.graph's default
    capture stream, so the same (device, stream, layout) key) must not share a scratch created inside the
    first capture: that scratch is cleared only by the first graph's replays.  Replay the second graph before
    the first has ever run, on a dirtied allocator, and compare both with the eager results.
    shared_pool: the second graph is captured into the first one's memory pool
    (torch.cuda.graph(..., pool=first.pool())), so a scratch of the first capture that the op's cache released
    could be handed to the second capture; the graphs are then replayed interleaved in capture order (the order
    torch requires of graphs sharing a pool), every output checked after every replay."""
    from dirt_amd import rasterise_ops
    ext = rasterise_ops._torch_ext()
    if impl == "ext":
        assert ext is not None

    def op(t0, t1, t2, ft, H, W, C):
        args = (t0, t1, t2, ft, None, H, W, C, 0, 0, False, False)
        return ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args)

    rasterise_ops.workspace_cache_clear(force=True)
    # fill the allocator's free blocks with garbage first, so that an uncleared scratch is not accidentally 0
    junk = [torch.full((1 << 22,), 0x01010101, dtype=torch.int32, device="cuda") for _ in range(16)]
    del junk
    scenes_ = [tuple(a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=s))
               for s in (90, 91)]
    B, H, W, C = scenes_[0][0].shape
    graphs, outs, refs, keep = [], [], [], []
    for bg, v, c, f in scenes_:
        t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
        ft = _gpu(f)
        g = torch.randn(bg.shape, device="cuda")
        keep.append((t, ft, g))  # a graph's inputs must outlive it (the loop rebinds t, ft, g)
        # the eager reference on the legacy default stream, the pattern users write.  Its output is released before
        # the capture: an autograd graph kept alive keeps the leaves' AccumulateGrad nodes, which remember the
        # default stream they were made on, and torch's engine then joins the capture stream with the default stream
        # inside the capture.  That ends in a segfault in torch.cuda.graph's capture_end on this stack with no
        # dirt_amd code at all (tools/debug/capture_control.py)
        px, _ = op(t[0], t[1], t[2], ft, H, W, C)
        refs.append((px.detach().clone(), [x.clone() for x in torch.autograd.grad(px, t, g)]))
        del px
        torch.cuda.synchronize()
        out = {}

        def step(t=t, ft=ft, g=g, out=out):
            px, _ = op(t[0], t[1], t[2], ft, H, W, C)
            out["px"] = px
            out["grads"] = torch.autograd.grad(px, t, g)

        # warm-up on a side stream (lazy autograd / allocator initialisation must not happen inside a capture), then
        # capture on torch.cuda.graph's class-wide default capture stream: both graphs share (device, stream, layout)
        s_ = torch.cuda.Stream()
        s_.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_):
            step()
        torch.cuda.current_stream().wait_stream(s_)
        torch.cuda.synchronize()
        out.clear()  # (the warm-up's autograd graph, made on s_, released before the capture for the same reason)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=graphs[0].pool() if shared_pool and graphs else None):
            step()
        graphs.append(graph)
        outs.append(out)
    torch.cuda.synchronize()
    ran = set()
    for k in ((0, 1, 0, 1) if shared_pool else (1, 0, 1, 0)):
        graphs[k].replay()
        torch.cuda.synchronize()
        ran.add(k)
        # (every graph replayed so far: a replay must not disturb another graph's outputs either)
        for j in sorted(ran):
            assert torch.equal(outs[j]["px"], refs[j][0]), "graph %d: pixels differ from the eager call" % j
            assert torch.equal(outs[j]["grads"][0], refs[j][1][0])
            for a, b in zip(outs[j]["grads"][1:], refs[j][1][1:]):
                torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()))
    del graphs
    rasterise_ops.workspace_cache_clear(force=True)


def test_captured_scratch_clear_is_ordered_in_the_graph():
    """A scratch created inside a capture is cleared by a node of that graph at every replay.  With the clear as a
    hipMemsetAsync node the bin counters were not clean at the next replay on this stack (they grew by 61,440 per
    replay, so every tile took the exact but slow all-records path, gpurun logs repro4_*.log of round 5); the clear is a
    kernel since round 5.  Replay a captured forward several times: the fullest slab stays at the eager count."""
    import ctypes
    from dirt_amd import _lib, rasterise_ops
    rasterise_ops.workspace_cache_clear(force=True)
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=92))
    B, H, W, C = bg.shape
    F = f.shape[1]
    t = [_gpu(a) for a in (bg, v, c, f)]

    def fwd():
        return rasterise_ops._RasteriseFunction.apply(t[0], t[1], t[2], t[3], None, H, W, C, 0, 0, False, False)

    lib = _lib.load()
    fn = lib.dirt_debug_bin_occupancy
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p] + \
        [ctypes.POINTER(ctypes.c_uint32)] * 3

    def max_count(scratch):
        mx, ov, slab = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _lib.check(fn(B, H, W, F, 0, scratch.data_ptr(), scratch.numel(), torch.cuda.current_stream().cuda_stream,
                      ctypes.byref(mx), ctypes.byref(ov), ctypes.byref(slab)))
        return mx.value, ov.value

    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        ref = fwd()[0].clone()
    torch.cuda.synchronize()
    eager = max_count(next(iter(rasterise_ops._workspace._d.values())))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = fwd()
    scratch = next(iter(next(iter(rasterise_ops._workspace._caps.values())).values()))
    for _ in range(4):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out[0], ref)
        assert max_count(scratch) == eager, (max_count(scratch), eager)
    del graph
    rasterise_ops.workspace_cache_clear(force=True)


def test_session_moves_between_streams():
    """RasteriseSession orders each call after the stream of its previous call: forward on one side stream,
    backward on another, no explicit synchronisation -- the gradients equal the single-stream ones."""
    from dirt_amd.session import RasteriseSession
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=20000, W=512, H=512, radius_px=12.0, seed=88))
    ts = [_gpu(a) for a in (bg, v, c, f)]
    g = torch.randn(bg.shape, device="cuda")
    sess = RasteriseSession(*bg.shape, v.shape[1], f.shape[1], device="cuda")
    sess.forward(*ts)
    ref = [x.clone() for x in sess.backward(g)]
    ref_px = sess.pixels.clone()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(s1):
            sess.forward(*ts)
        with torch.cuda.stream(s2):
            out = sess.backward(g)
            res = [x.clone() for x in out] + [sess.pixels.clone()]
        torch.cuda.current_stream().wait_stream(s2)
        torch.cuda.synchronize()
        assert torch.equal(res[3], ref_px)
        assert torch.equal(res[0], ref[0])
        for a, b in zip(res[1:3], ref[1:]):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()))


@pytest.mark.parametrize("want_gbuf", [False, True])
def test_cpp_autograd_op_matches_python_function(want_gbuf):
    """The public op runs the C++ autograd function (_dirt_torch, dirt_amd/csrc/torch_op.cpp) when built;
    the Python torch.autograd.Function (_RasteriseFunction) is the same op over the same C ABI.  Both give
    bit-identical forwards and the same gradients, on a fused small scene and a binned one, with a
    retained graph's second backward."""
    from dirt_amd import rasterise_ops
    ext = rasterise_ops._torch_ext()
    assert ext is not None, "the C++ extension dirt_amd/_dirt_torch*.so is not built"
    for sc in (scenes.cube_scene(), scenes.random_triangles(F=1500, W=128, H=96, radius_px=10.0, seed=90,
                                                             perspective=True)):
        bg, v, c, f = (a[None] for a in sc)
        B, H, W, C = bg.shape
        g = torch.randn(bg.shape, device="cuda")
        res = []
        for impl in ("ext", "py"):
            t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
            args = (t[0], t[1], t[2], _gpu(f), None, H, W, C, 0, 0, want_gbuf, False)
            outs = ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args)
            g1 = torch.autograd.grad(outs[0], t, g, retain_graph=True)
            g2 = torch.autograd.grad(outs[0], t, g)
            res.append(([o.detach().clone() for o in outs], g1, g2))
        (oe, ge1, ge2), (op, gp1, gp2) = res
        assert len(oe) == len(op) == (5 if want_gbuf else 2)
        for a, b in zip(oe, op):
            assert torch.equal(a, b)
        for a, b in zip(ge1 + ge2, gp1 + gp1):
            assert torch.equal(a, b) if a.shape == bg.shape else True
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()) + 1e-30)


def test_public_op_without_gradients():
    """Inputs that need no gradient, and calls under torch.no_grad(): no graph is recorded, no gradient
    buffers are zero-filled, the forward is the same."""
    import dirt_amd
    bg, v, c, f = scenes.random_triangles(F=800, W=80, H=64, radius_px=9.0, seed=91)
    ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
    px = dirt_amd.rasterise(_gpu(bg), _gpu(v), _gpu(c), _gpu(f))
    assert not px.requires_grad
    np.testing.assert_array_equal(px.cpu().numpy(), ref[0])
    t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
    with torch.no_grad():
        px = dirt_amd.rasterise(t[0], t[1], t[2], _gpu(f))
    assert not px.requires_grad
    np.testing.assert_array_equal(px.cpu().numpy(), ref[0])
    px = dirt_amd.rasterise(t[0].detach(), t[1], t[2].detach(), _gpu(f))  # only vertices need a gradient
    (gv,) = torch.autograd.grad(px, [t[1]], torch.ones_like(px))
    assert torch.isfinite(gv).all()


def _bin_occupancy(B, H, W, F, scratch, nbytes):
    import ctypes
    from dirt_amd import _lib
    lib = _lib.load()
    fn = lib.dirt_debug_bin_occupancy
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p] + \
        [ctypes.POINTER(ctypes.c_uint32)] * 3
    mx, ov, slab = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(fn(B, H, W, F, 0, scratch.data_ptr(), nbytes, torch.cuda.current_stream().cuda_stream,
                  ctypes.byref(mx), ctypes.byref(ov), ctypes.byref(slab)))
    return mx.value, ov.value, slab.value


@pytest.mark.parametrize("B", [8, 64])
def test_clustered_mesh_at_config5_batch_shape(B):
    """a mesh crowded into the centre 1/16 of every frame (20k faces per frame, 1024^2) at config
    5's per-rank batch (8 frames) and at all 64 frames on one GPU: no coarse-tile slab overflows at the
    default capacity (the 2^29-entry budget keeps F + F/4 + 64 per slab at B = 64), and the result is
    bit-exact against the oracle (frames 0 and B-1 checked for gradients)."""
    from dirt_amd.session import RasteriseSession
    frames = [scenes.random_triangles(F=20000, W=1024, H=1024, seed=200 + b, spread=0.25) for b in range(B)]
    bg, v, c, f = (np.stack([fr[k] for fr in frames]) for k in range(4))
    sess = RasteriseSession(B, 1024, 1024, 3, v.shape[1], f.shape[1], device="cuda")
    g = np.random.default_rng(5).standard_normal(bg.shape).astype(np.float32)
    sess.forward(*(_gpu(a) for a in (bg, v, c, f)))
    mx, ov, slab = _bin_occupancy(B, 1024, 1024, f.shape[1], sess.scratch, sess.scratch_bytes)
    assert slab >= 20000 + 20000 // 4 + 64 and ov == 0 and 0 < mx <= slab, (mx, ov, slab)
    gbg, gv, gc = (t.cpu().numpy() for t in sess.backward(_gpu(g)))
    px, gb = sess.pixels.cpu().numpy(), sess.gbuffer.cpu().numpy()
    for b in sorted({0, B - 1}):
        sl = slice(b, b + 1)
        rpx, rgb, _ = oracle.rasterise_fwd(bg[sl], v[sl], c[sl], f[sl])
        np.testing.assert_array_equal(gb[sl], rgb)
        np.testing.assert_array_equal(px[sl], rpx)
        rgv, rgc, rgbg = oracle.rasterise_bwd(v[sl], c[sl], f[sl], rpx, g[sl], rgb)
        np.testing.assert_array_equal(gbg[sl], rgbg)
        for a, r in ((gv[sl], rgv), (gc[sl], rgc)):
            err = np.abs(a - r)
            assert (err <= 1e-4 * np.abs(r) + 1e-5 * np.abs(r).max()).all()
