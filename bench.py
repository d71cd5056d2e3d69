#!/usr/bin/env python3
"""Benchmark of the dirt rasterise hot path (forward + backward) on MI355X.

Metric (BASELINE.json): Mpixels/s fwd+bwd at 1024x1024, 50k random triangles (config 3).
One step = dirt rasterise forward + registered backward over one synthetic frame per rank
(SURVEY 8d distribution, seed = rank), inputs resident in HBM.  N>1: one process per GPU, frames
sharded across ranks with no data-path collective (weak scaling); value = all ranks' pixels / max time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0).  Extra keys: roofline (dominant kernel, HIP-event timed), cpu_baseline
(the CPU oracle on the box's host cores, rank 0 at N=1), kernels (per-kernel average microseconds).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip-level table)
# measured HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, rocprofv3 --pmc passes of this bench at c3;
# produced by tools/gpu_traffic.sh + tools/pmc_traffic.py, committed with the round's profiles)
# (the newest round's file; it names the tree and the box it was measured on, `measured_on`)
TRAFFIC_JSON = next((p for p in (os.path.join(ROOT, "profiles", r, "traffic.json") for r in ("r06", "r05", "r04"))
                     if os.path.exists(p)), os.path.join(ROOT, "profiles", "r06", "traffic.json"))

CONFIGS = {
    # name: (B per rank, H, W, C, F, radius_px)
    "c3": (1, 1024, 1024, 3, 50000, 16.0),
    "c5": (8, 1024, 1024, 3, 20000, 16.0),  # 64 frames over 8 GPUs -> 8 per rank
    "c3_r64": (1, 1024, 1024, 3, 50000, 64.0),
    # config 3 frames eight to a launch (profiling: the kernels' steady state, no single-round ramp or drain tail)
    "c3x8": (8, 1024, 1024, 3, 50000, 16.0),
}


def alg_bytes(B, H, W, C, V, F):
    """Algorithmic HBM bytes, SURVEY 8(d): the tensor I/O of the op's C ABI, intermediates (records, bins, the
    g-buffer) excluded.  fwd = 16V + 12F + 4CV + 4CHW (background) + 4CHW (pixels); bwd = 16V + 12F + 4CV (inputs)
    + 4CHW (pixels) + 4CHW (grad_pixels) + 16V + 4CV (gradient outputs) + 4CHW (grad_background) -- config 3:
    29.96 + 46.75 MB.  Per kernel: the backward is the one grad launch (all of bwd); the forward's split is setup =
    vertices + faces, raster = colours + background + pixels."""
    hwc = 4 * C * H * W
    fwd = B * (16 * V + 12 * F + 4 * C * V + 2 * hwc)
    bwd = B * (16 * V + 12 * F + 4 * C * V + 2 * hwc + 16 * V + 4 * C * V + hwc)
    k = {
        "setup_kernel": B * (16 * V + 12 * F),
        "raster_kernel": B * (4 * C * V + 2 * hwc),
        "grad_kernel": bwd,
    }
    return k, fwd, bwd


def make_inputs(cfg, rank, device):
    import scenes
    B, H, W, C, F, r = cfg
    frames = [scenes.random_triangles(F=F, W=W, H=H, C=C, radius_px=r, seed=rank * B + b) for b in range(B)]
    host = [np.stack([fr[k] for fr in frames]) for k in range(4)]
    dev = [torch.from_numpy(a).to(device) for a in host]
    g = np.random.default_rng(10_000 + rank).standard_normal(host[0].shape).astype(np.float32)
    return host, dev, torch.from_numpy(g).to(device), g


def host_cpu_info():
    """What the CPU baseline ran on: the threads it used, the box's online CPUs and this process's affinity,
    and the lscpu model name."""
    model = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.lower().startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:  # lscpu absent: report what Python knows
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return {"cpu_model": model, "nproc_online": os.cpu_count(), "affinity_cpus": affinity}


def cpu_share():
    """Evidence for the CPU share the baseline runs on: the cgroup CPU quota (cgroup v2 cpu.max, v1
    cfs_quota / cfs_period), the cpuset, OMP_NUM_THREADS as the box sets it, and the CPUs online."""
    out = {"OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "nproc_online": os.cpu_count()}
    for key, path in (("cgroup_cpu_max", "/sys/fs/cgroup/cpu.max"),
                      ("cgroup_cpuset_effective", "/sys/fs/cgroup/cpuset.cpus.effective"),
                      ("cgroup_v1_cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"),
                      ("cgroup_v1_cfs_period_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            out[key] = open(path).read().strip()
        except OSError:
            pass
    q = out.get("cgroup_cpu_max", "").split()
    if len(q) == 2 and q[0] != "max":
        out["cgroup_cpu_quota_cpus"] = round(int(q[0]) / int(q[1]), 2)
    return out


def cpu_threads():
    """Every host core this job may use: the CPU share the pool grants one GPU's job (OMP_NUM_THREADS, which
    the GPU box sets; the box's rules size worker pools to that share), else the process's affinity mask."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        return env
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(host, grad_host, budget_s=10.0, max_reps=20):
    from oracle import oracle
    nthreads = cpu_threads()
    bg, v, c, f = host
    B, H, W, C = bg.shape
    times = []
    t_start = time.perf_counter()
    while len(times) < max_reps and (time.perf_counter() - t_start < budget_s or len(times) < 1):
        t0 = time.perf_counter()
        px, gb, _ = oracle.rasterise_fwd(bg, v, c, f, nthreads=nthreads)
        grads = oracle.rasterise_bwd(v, c, f, px, grad_host, gb, nthreads=nthreads)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    out = {"value": B * H * W / t / 1e6, "unit": "Mpixels/s", "cores": nthreads, "kind": "port",
           "sample": "%d x full config frame(s) (%dx%dx%d, F=%d) fwd+bwd, median of %d reps, oracle/dirt_oracle.c "
                     "OpenMP, %d threads" % (B, H, W, C, f.shape[1], len(times), nthreads),
           "ms_per_frame": t * 1e3 / B}
    out.update(host_cpu_info())
    out["cpu_share"] = cpu_share()
    return out, (px, gb) + tuple(grads)


def parity(sess, ref):
    """The metric's 'grad max-abs-err vs ref': the benchmarked step's outputs against the CPU oracle on the
    same frame (forward bit-exact; gradients within the DESIGN.md section 5 tolerance)."""
    px, gb, rgv, rgc, rgbg = ref
    out = {"pixels_max_abs_err": float(np.abs(sess.pixels.cpu().numpy() - px).max()),
           "gbuffer_mismatches": int((sess.gbuffer.cpu().numpy() != gb).sum())}
    for name, a, b in (("grad_vertices", sess.grad_vertices, rgv), ("grad_vertex_colors", sess.grad_vertex_colors, rgc),
                       ("grad_background", sess.grad_background, rgbg)):
        e = np.abs(a.cpu().numpy() - b)
        out[name + "_max_abs_err"] = float(e.max())
        out[name + "_max_abs_ref"] = float(np.abs(b).max())
        tol = 1e-4 * np.abs(b) + 1e-5 * max(float(np.abs(b).max()), 1e-30)
        out[name + "_within_tol"] = bool((e <= tol).all())
    return out


def graph_of(fn, n, stream):
    """Capture n calls of fn into one HIP graph on `stream` (warmed on the same stream first, so cached
    workspaces keyed by stream are hit instead of allocated inside the capture).  `stream` first waits for
    the current stream: a session's buffers are stream-ordered, and steps still in flight there must not
    overlap the warm-up call's reuse of them."""
    stream.wait_stream(torch.cuda.current_stream(stream.device))
    with torch.cuda.stream(stream):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(n):
            fn()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    return g


def timed(run, n_calls, barrier, world, device, shared):
    """Run `run` n_calls times between barrier + synchronize on both sides; max over ranks (seconds)."""
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_calls):
        run()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a HIP graph")
    ap.add_argument("--graph-steps", type=int, default=200,
                    help="steps captured per HIP graph (each replay runs that many complete steps; default: all "
                         "timed steps up to 200 in one graph, since every replay boundary costs ~24 us)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--profile-steps", type=int, default=50)
    ap.add_argument("--rotate", type=int, default=4,
                    help="extra leg: rotate this many distinct frames (inputs, outputs, workspaces) so the step's "
                         "working set exceeds the 256 MiB Infinity Cache; 0 = skip")
    ap.add_argument("--no-api-leg", action="store_true", help="skip the public rasterise_batch + autograd leg")
    ap.add_argument("--no-gather-leg", action="store_true", help="N > 1: skip the RCCL all-gather leg")
    ap.add_argument("--no-recompute-leg", action="store_true", help="skip the recompute-backward leg")
    ap.add_argument("--min-warm-ms", type=float, default=200.0,
                    help="after the warmup steps, keep running the step untimed for this long (GPU clock ramp); "
                         "0 = off")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # DIRT_BENCH_SHARED_GPU=1: rehearsal of the N-rank path on a box with fewer GPUs than ranks (ranks share
    # cuda:LOCAL_RANK % count, collectives over gloo); the driver's multi-GPU runs leave it unset (RCCL)
    shared = os.environ.get("DIRT_BENCH_SHARED_GPU") == "1"
    if shared:
        local_rank %= max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    from dirt_amd import _lib
    from dirt_amd.session import RasteriseSession

    cfg = CONFIGS[args.config]
    B, H, W, C, F, _r = cfg
    V = 3 * F
    host, (bg, v, c, f), grad, grad_host = make_inputs(cfg, rank, device)
    sess = RasteriseSession(B, H, W, C, V, F, device=device)
    cap_stream = torch.cuda.Stream(device)

    def step():
        sess.forward(bg, v, c, f)
        sess.backward(grad)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    # the timed loop runs exactly args.steps complete steps: full graph replays of gs steps each, the
    # remainder eagerly
    gs = 1 if args.no_graph else max(1, min(args.graph_steps, args.steps))
    n_replays, n_rest = divmod(args.steps, gs)
    if args.no_graph:
        n_replays, n_rest = args.steps, 0
        run = step
    else:
        run = graph_of(step, gs, cap_stream).replay
    # Clock warm-up (untimed, reported in the line): the GPU raises its clock only under sustained load, and
    # W short steps (~0.3 ms at W = 5) end before it has, so a 20-step timed window would measure the ramp
    # (profiles/r03/driver_flags: kernels 8 % slower at K = 20, W = 5 than after a long run).  The same
    # step keeps running untimed until --min-warm-ms of it has passed; the timed region is unchanged.
    warm_steps, t_w0 = 0, time.perf_counter()
    while args.min_warm_ms > 0 and (time.perf_counter() - t_w0) * 1e3 < args.min_warm_ms:
        run()
        warm_steps += gs if not args.no_graph else 1
        torch.cuda.synchronize()
    clock_warm = {"untimed_steps": warm_steps, "ms": round((time.perf_counter() - t_w0) * 1e3, 1)}

    def timed_loop():
        for _ in range(n_replays):
            run()
        for _ in range(n_rest):
            step()

    elapsed = timed(timed_loop, 1, barrier, world, device, shared)
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * B * H * W * args.steps / elapsed / 1e6

    # per-kernel HIP-event timing (same kernels, eager launches, outside the timed loop)
    def kernel_times(fn, n):
        _lib.profile_enable(True)
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        prof = _lib.profile_read()
        _lib.profile_enable(False)
        return {k: (ms / cnt * 1e3 if cnt else 0.0) for k, (cnt, ms) in prof.items()}

    kern_us = kernel_times(step, args.profile_steps)
    kbytes, fwd_b, bwd_b = alg_bytes(B, H, W, C, V, F)

    def pass_times_graph(n=50):
        """Each pass inside a replayed graph, without the per-launch gap that the event pair around an eager
        launch includes: HIP events around one replay of n forwards (setup + raster) and of n backwards (grad
        alone: the backward accumulates, so repeating it is the same work).  rocprofv3 --kernel-trace reports
        the same durations (profiles/r03/ev2_kernel_stats_graph.csv)."""
        out = {}
        for name, fn in (("fwd_setup_plus_raster", lambda: sess.forward(bg, v, c, f)),
                         ("bwd_grad", lambda: sess.backward(grad))):
            g = graph_of(fn, n, cap_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()  # (replay() launches on the current stream)
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) * 1e3 / n
            del g
        step()  # (the session's buffers hold one consistent forward + backward again)
        torch.cuda.synchronize()
        return out

    pass_us = None
    if not args.no_graph:
        try:
            pass_us = pass_times_graph()
        except Exception as e:  # noqa: BLE001 -- informative field only
            print("graph pass timing failed: %s" % e, file=sys.stderr)
            torch.cuda.synchronize()

    def grad_dispatch_us(n=50):
        """The backward kernel's duration from hipExtLaunchKernel's dispatch events (dirt_debug_bwd_dispatch_ms: the
        product instantiation, `n` launches on the bench stream, each timed at its own dispatch) -- what rocprofv3
        --kernel-trace reports; the graph pass above and the eager event pairs add each launch's dependent-launch gap."""
        import ctypes
        lib = _lib.load()
        fn = lib.dirt_debug_bwd_dispatch_ms
        P = ctypes.c_void_p
        fn.argtypes = [P, P, P, P] + [ctypes.c_int] * 6 + [P, P, P, ctypes.c_int, P, ctypes.POINTER(ctypes.c_float)]
        fn.restype = ctypes.c_int
        ms = ctypes.c_float(0.0)
        torch.cuda.synchronize()
        _lib.check(fn(sess.pixels.data_ptr(), grad.data_ptr(), sess.gbuffer.data_ptr(), sess.saved.data_ptr(),
                      B, H, W, C, V, F, sess.grad_vertices.data_ptr(), sess.grad_vertex_colors.data_ptr(),
                      sess.grad_background.data_ptr(), n, torch.cuda.current_stream().cuda_stream, ctypes.byref(ms)))
        step()  # (the session's buffers hold one consistent forward + backward again)
        torch.cuda.synchronize()
        return ms.value * 1e3

    disp_us = None
    if C == 3:
        try:
            disp_us = grad_dispatch_us()
        except Exception as e:  # noqa: BLE001 -- informative field only
            print("dispatch timing failed: %s" % e, file=sys.stderr)
            torch.cuda.synchronize()
    # The roofline kernel is the backward scatter (grad_kernel), the kernel the north star states its bandwidth
    # target on (the raster is the longer launch since round 6, `dominant_kernel_by_events`).
    # achieved = SURVEY 8(d)'s backward bytes (46.75 MB at c3) / the kernel's average duration: hipExtLaunchKernel's
    # dispatch events over 50 launches on the bench stream (what rocprofv3 --kernel-trace reports), else HIP events
    # around one replay of a graph of 50 backward launches (`avg_us_graph`, which adds the dependent-launch gap), else
    # the eager event pairs (`avg_us_events`).
    dom = "grad_kernel"
    dom_events = max((k for k in kern_us if k in kbytes), key=lambda k: kern_us[k])
    dur_us = disp_us if disp_us else (pass_us["bwd_grad"] if pass_us else kern_us[dom])
    achieved = kbytes[dom] / (dur_us * 1e-6) / 1e9
    traffic = measured_on = None
    if args.config == "c3" and os.path.exists(TRAFFIC_JSON):
        tj = json.load(open(TRAFFIC_JSON))
        hit = [v for k, v in tj.get("kernels", {}).items() if k.split("<")[0] == dom]
        if hit:
            traffic = hit[0]["traffic_bytes"]
            measured_on = tj.get("measured_on")
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": os.path.relpath(TRAFFIC_JSON, ROOT) if traffic is not None else None,
                "traffic_measured_on": measured_on,
                "alg_bytes_per_launch": kbytes[dom], "alg_bytes_definition": "SURVEY 8(d) bwd",
                "avg_us": round(dur_us, 2),
                "avg_us_source": ("hipExtLaunchKernel dispatch events, 50 launches" if disp_us else
                                  "graph of 50 launches, HIP events" if pass_us else "eager HIP event pairs"),
                "avg_us_graph": round(pass_us["bwd_grad"], 2) if pass_us else None,
                "avg_us_events": round(kern_us[dom], 2), "dominant_kernel_by_events": dom_events,
                "op_frac": round((fwd_b + bwd_b) / (ms_per_step * 1e-3 / world) / 1e9 / HBM_PEAK_GBS, 4)}
    # the op's algorithmic bytes over each pass's kernel time (fwd = setup + raster, bwd =
    # grad), and the measured HBM bytes (rocprof PMC, traffic.json) of the dominant kernel over its time --
    # the north-star's "HBM bandwidth on the backward scatter" is stated on measured bytes
    t_fwd = kern_us.get("setup_kernel", 0.0) + kern_us.get("raster_kernel", 0.0)
    t_bwd = kern_us.get("grad_kernel", 0.0)
    if t_fwd > 0:
        roofline["fwd_frac"] = round(fwd_b / (t_fwd * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    if t_bwd > 0:
        roofline["bwd_frac"] = round(bwd_b / (t_bwd * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    if traffic is not None:
        roofline["traffic_frac"] = round(traffic / (dur_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    if pass_us:
        # the same fractions on the passes' in-graph times (a graph of back-to-back launches: each launch's
        # dependent-launch gap included)
        roofline["graph_pass_us"] = {k: round(u, 2) for k, u in pass_us.items()}
        roofline["fwd_frac_graph"] = round(fwd_b / (pass_us["fwd_setup_plus_raster"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        roofline["bwd_frac_graph"] = round(bwd_b / (pass_us["bwd_grad"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        roofline["grad_kernel_frac_graph"] = round(kbytes["grad_kernel"] / (pass_us["bwd_grad"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        if traffic is not None and dom == "grad_kernel":
            roofline["traffic_frac_graph"] = round(traffic / (pass_us["bwd_grad"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)

    legs = {}

    def leg(name, fn):
        """Run one extra leg; a failure is reported in the JSON line instead of ending the run (the headline
        `value` above is already measured)."""
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- any leg failure is data, not a reason to lose the line
            legs[name] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}
            torch.cuda.synchronize()

    def api_leg():
        import dirt_amd
        from dirt_amd import rasterise_ops
        # every step a full forward, as in training (the optimizer changes the vertices each step): the shared-geometry
        # cache off, which would otherwise serve this leg's repeated, unmodified geometry from its first render
        share_prev = rasterise_ops.set_geometry_sharing(False)
        try:
            api_leg_measure(dirt_amd, rasterise_ops)
        finally:
            rasterise_ops.set_geometry_sharing(share_prev)

    def api_leg_measure(dirt_amd, rasterise_ops):
        bg_r, v_r, c_r = (t.clone().requires_grad_(True) for t in (bg, v, c))

        def api_step():
            px = dirt_amd.rasterise_batch(bg_r, v_r, c_r, f)
            torch.autograd.grad(px, [bg_r, v_r, c_r], grad)

        # the headline's clock warm-up (the eager op is host-bound, so the GPU idles between launches and its clock
        # falls back quickly), then at least 200 timed eager steps in chunks of 20: the rate over all of them
        # plus the median and spread of the chunks (20 steps were noise-dominated)
        t_w = time.perf_counter()
        while (time.perf_counter() - t_w) * 1e3 < max(args.min_warm_ms, 50.0):
            api_step()
        torch.cuda.synchronize()
        chunk = 20
        n_chunks = max(10, -(-args.steps // chunk))
        chunk_s = [timed(api_step, chunk, barrier, world, device, shared) for _ in range(n_chunks)]
        n_api = chunk * n_chunks
        t_eager = sum(chunk_s)
        rates = sorted(world * B * H * W * chunk / t / 1e6 for t in chunk_s)
        g_api = graph_of(api_step, 1, cap_stream)
        t_graph = timed(g_api.replay, n_api, barrier, world, device, shared)
        del g_api
        # the same with 20 steps per graph (each step's fresh outputs come from the graph's pool, ~75 MB per step
        # at c3): the replay boundary (~24 us) amortised as in the headline's 200-step graphs
        g_api20 = graph_of(api_step, 20, cap_stream)
        n20 = max(2, n_api // 20)
        t_graph20 = timed(g_api20.replay, n20, barrier, world, device, shared)
        del g_api20
        # for reference: the same eager loop with the cache on (an inference-like repeat of one geometry: every
        # forward after the first runs the resolve alone); not a training step
        rasterise_ops.set_geometry_sharing(True)
        t_sh = sum(timed(api_step, chunk, barrier, world, device, shared) for _ in range(n_chunks))
        rasterise_ops.set_geometry_sharing(False)
        legs["api_autograd"] = {
            "what": "dirt_amd.rasterise_batch(...) + torch.autograd.grad per step (reference surface "
                    "dirt/rasterise_ops.py:57-88), fresh outputs per call, cached scratch, every forward a full one "
                    "(shared-geometry cache off; eager_shared_geometry_mpix_s: the same loop with it on)",
            "eager_mpix_s": round(world * B * H * W * n_api / t_eager / 1e6, 1),
            "eager_ms_per_step": round(t_eager * 1e3 / n_api, 4),
            "eager_steps": n_api,
            "eager_chunks_mpix_s": {"chunk_steps": chunk, "median": round(float(np.median(rates)), 1),
                                    "min": round(rates[0], 1), "max": round(rates[-1], 1)},
            "graph_mpix_s": round(world * B * H * W * n_api / t_graph / 1e6, 1),
            "graph_ms_per_step": round(t_graph * 1e3 / n_api, 4),
            "graph20_mpix_s": round(world * B * H * W * n20 * 20 / t_graph20 / 1e6, 1),
            "graph20_ms_per_step": round(t_graph20 * 1e3 / (n20 * 20), 4),
            "geometry_sharing": False,
            "eager_shared_geometry_mpix_s": round(world * B * H * W * n_api / t_sh / 1e6, 1),
            "impl": "C++ autograd function (_dirt_torch)" if dirt_amd.rasterise_ops._torch_ext() is not None
                    else "Python torch.autograd.Function"}

    # ---- leg: the public op surface (dirt_amd.rasterise_batch + torch.autograd), eager and graph-captured
    if not args.no_api_leg:
        leg("api_autograd", api_leg)

    def recompute_leg():
        """The single-output op (dirt_rasterise_fwd_stash + the registered gradient dirt_rasterise_bwd_recompute on
        the op's workspace), graph-captured like the headline step, against the stateful session step; and the
        same gradient when the workspace does not hold the geometry (always recomputed: setup + bins +
        coverage-only raster + backward kernel)."""
        lib = _lib.load()
        n_ws = _lib.recompute_workspace_size(B, H, W, C, V, F)
        ws = torch.zeros((n_ws,), dtype=torch.uint8, device=device)
        ws2 = torch.zeros((n_ws,), dtype=torch.uint8, device=device)
        px = torch.empty((B, H, W, C), device=device)
        gv = torch.empty((B, V, 4), device=device)
        gc = torch.empty((B, V, C), device=device)
        gbg = torch.empty((B, H, W, C), device=device)

        def rc_bwd(w, flags, pixels=px):
            stream = torch.cuda.current_stream(device).cuda_stream
            _lib.check(lib.dirt_rasterise_bwd_recompute(
                bg.data_ptr(), v.data_ptr(), c.data_ptr(), f.data_ptr(), pixels.data_ptr(), grad.data_ptr(),
                B, H, W, C, V, F, gv.data_ptr(), gc.data_ptr(), gbg.data_ptr(), w.data_ptr(), n_ws, flags, stream))

        def stash_step():
            stream = torch.cuda.current_stream(device).cuda_stream
            _lib.check(lib.dirt_rasterise_fwd_stash(bg.data_ptr(), v.data_ptr(), c.data_ptr(), f.data_ptr(), B, H, W,
                                                    C, V, F, px.data_ptr(), ws.data_ptr(), n_ws,
                                                    _lib.FWD_SCRATCH_CLEAN, stream))
            rc_bwd(ws, _lib.BWD_SCRATCH_CLEAN)

        def miss_step():
            # (flags 0: the workspace is not vouched clean, so its stash header is reset -- always a recomputation)
            sess.forward(bg, v, c, f)
            rc_bwd(ws2, 0, sess.pixels)

        out = {}
        for name, fn in (("stash", stash_step), ("no_stash", miss_step)):
            for _ in range(5):
                fn()
            n_rc = max(20, args.steps)
            g_rc = graph_of(fn, min(n_rc, 200), cap_stream) if not args.no_graph else None
            reps = max(1, n_rc // min(n_rc, 200)) if g_rc else n_rc
            t_rc = timed(g_rc.replay if g_rc else fn, reps, barrier, world, device, shared)
            steps_rc = reps * (min(n_rc, 200) if g_rc else 1)
            out[name] = (t_rc, steps_rc)
            del g_rc
        st = _lib.stash_state(B, H, W, C, V, F, ws.data_ptr(), n_ws, torch.cuda.current_stream(device).cuda_stream)
        kr = kernel_times(lambda: rc_bwd(ws, _lib.BWD_SCRATCH_CLEAN), args.profile_steps)
        (t_s, n_s), (t_m, n_m) = out["stash"], out["no_stash"]
        legs["recompute_bwd"] = {
            "what": "the single-output op per step: dirt_rasterise_fwd_stash + its registered gradient "
                    "dirt_rasterise_bwd_recompute on the op's workspace (the geometry compared bitwise on the device; "
                    "unchanged, so the recomputation is skipped); no_stash: the same gradient recomputing setup + "
                    "bins + coverage-only raster every step",
            "mpix_s": round(world * B * H * W * n_s / t_s / 1e6, 1),
            "ms_per_step": round(t_s * 1e3 / n_s, 4),
            "stateful_ms_per_step": round(ms_per_step, 4),
            "extra_us_per_step": round((t_s / n_s - ms_per_step * 1e-3) * 1e6, 2),
            "stash_last_missed": st["last_missed"],
            "no_stash_mpix_s": round(world * B * H * W * n_m / t_m / 1e6, 1),
            "no_stash_extra_us_per_step": round((t_m / n_m - ms_per_step * 1e-3) * 1e6, 2),
            "bwd_kernels_us": {k: round(u, 2) for k, u in kr.items()}}
        del ws, ws2
        step()
        torch.cuda.synchronize()

    # ---- leg: the single-output op's recompute-mode gradient (its extra cost over the stateful step)
    if not args.no_recompute_leg:
        leg("recompute_bwd", recompute_leg)

    def cold_leg():
        R = args.rotate
        rot = []
        for k in range(R):
            hk, dk, gk, _ = make_inputs(cfg, rank + 1000 * (k + 1), device)
            rot.append((RasteriseSession(B, H, W, C, V, F, device=device), dk, gk))
        per_frame = sum(t.numel() * t.element_size() for t in rot[0][1]) + rot[0][2].numel() * 4
        per_frame += sum(t.numel() * t.element_size() for t in (rot[0][0].pixels, rot[0][0].gbuffer, rot[0][0].saved,
                                                             rot[0][0].grad_vertices, rot[0][0].grad_vertex_colors,
                                                             rot[0][0].grad_background))
        idx = [0]

        def rot_step():
            se, (bg_k, v_k, c_k, f_k), g_k = rot[idx[0] % R]
            idx[0] += 1
            se.forward(bg_k, v_k, c_k, f_k)
            se.backward(g_k)

        for _ in range(2 * R):
            rot_step()
        n_rot = max(R, (args.steps // R) * R)
        g_rot = graph_of(lambda: [rot_step() for _ in range(R)], 1, cap_stream) if not args.no_graph else None
        t_rot = timed((g_rot.replay if g_rot else lambda: [rot_step() for _ in range(R)]), n_rot // R, barrier,
                      world, device, shared)
        kr = kernel_times(rot_step, max(args.profile_steps // R, 1) * R)
        legs["cold_cache"] = {
            "what": "%d distinct frames rotated step by step (inputs, outputs and workspaces), %.0f MB touched per "
                    "rotation > 256 MiB Infinity Cache" % (R, R * per_frame / 1e6),
            "mpix_s": round(world * B * H * W * n_rot / t_rot / 1e6, 1),
            "ms_per_step": round(t_rot * 1e3 / n_rot, 4),
            "kernels_us": {k: round(u, 2) for k, u in kr.items()},
            "grad_kernel_frac": round(kbytes["grad_kernel"] / (kr["grad_kernel"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        del g_rot, rot

    # ---- leg: rotating distinct frames, working set past the 256 MiB Infinity Cache (cold HBM)
    if args.rotate > 1:
        leg("cold_cache", cold_leg)

    def gather_leg():
        from dirt_amd.sharding import gather_frames_async
        batch = world * B
        for _ in range(3):
            gather_frames_async(sess.pixels, batch)[1]()
        n_g = max(10, args.steps // 4)
        t_g = timed(lambda: gather_frames_async(sess.pixels, batch)[1](), n_g, barrier, world, device, shared)
        # the single-consumer variant: every frame to rank 0 only
        from dirt_amd.sharding import gather_frames_to
        gather_frames_to(sess.pixels, batch, dst=0)
        t_root = timed(lambda: gather_frames_to(sess.pixels, batch, dst=0), n_g, barrier, world, device, shared)
        # reduced-precision wire format: bf16 pixels, half the xGMI bytes
        gather_frames_async(sess.pixels, batch, dtype=torch.bfloat16)[1]()
        t_bf = timed(lambda: gather_frames_async(sess.pixels, batch, dtype=torch.bfloat16)[1](), n_g, barrier, world,
                     device, shared)
        t_root_bf = timed(lambda: gather_frames_to(sess.pixels, batch, dst=0, dtype=torch.bfloat16), n_g, barrier,
                          world, device, shared)
        # pipelined: step k's frames move while step k+1 renders (two sessions, so a frame being gathered
        # is never overwritten; the step that reuses a session first waits for its gather)
        sess2 = RasteriseSession(B, H, W, C, V, F, device=device)
        pair = (sess, sess2)
        pend = [None, None]

        mode = {"fn": lambda px: gather_frames_async(px, batch)}

        def piped(k):
            se = pair[k & 1]
            if pend[k & 1] is not None:
                pend[k & 1][0].wait()
            se.forward(bg, v, c, f)
            se.backward(grad)
            pend[k & 1] = mode["fn"](se.pixels)

        for k in range(4):
            piped(k)
        for p_ in pend:
            p_[1]()
        pend[:] = [None, None]
        ctr = [0]

        def piped_run():
            piped(ctr[0])
            ctr[0] += 1

        def piped_all():
            for _ in range(args.steps):
                piped_run()
            for p_ in pend:
                if p_ is not None:
                    p_[1]()

        t_p = timed(piped_all, 1, barrier, world, device, shared)
        from dirt_amd.sharding import gather_frames_to_async
        piped_modes = {}
        for name, fn in (("bf16_all_gather", lambda px: gather_frames_async(px, batch, dtype=torch.bfloat16)),
                         ("f32_to_rank0", lambda px: gather_frames_to_async(px, batch, dst=0)),
                         ("bf16_to_rank0", lambda px: gather_frames_to_async(px, batch, dst=0, dtype=torch.bfloat16))):
            mode["fn"] = fn
            for k in range(4):
                piped(k)
            for p_ in pend:
                p_[1]()
            pend[:] = [None, None]
            t_m = timed(piped_all, 1, barrier, world, device, shared)
            piped_modes[name] = {"value_with_gather": round(world * B * H * W * args.steps / t_m / 1e6, 1),
                                 "ms_per_step": round(t_m * 1e3 / args.steps, 4)}
        recv = (world - 1) * B * H * W * C * 4
        legs["gather"] = {
            "what": "all_gather_into_tensor of every rank's pixels [%d,%d,%d,%d] over %s per step" %
                    (B, H, W, C, "gloo (shared-GPU rehearsal)" if shared else "RCCL / xGMI"),
            "gather_ms": round(t_g * 1e3 / n_g, 4),
            "gather_to_rank0_ms": round(t_root * 1e3 / n_g, 4),
            "recv_bytes_per_rank": recv,
            "recv_GBps_per_rank": round(recv / (t_g / n_g) / 1e9, 1),
            "gather_bf16_ms": round(t_bf * 1e3 / n_g, 4),
            "gather_to_rank0_bf16_ms": round(t_root_bf * 1e3 / n_g, 4),
            "value_with_gather": round(world * B * H * W * args.steps / t_p / 1e6, 1),
            "ms_per_step_with_gather": round(t_p * 1e3 / args.steps, 4),
            "pipelined_variants": piped_modes}

    # ---- leg (N > 1): the output all-gather over RCCL / xGMI, alone and overlapped with the next step
    if world > 1 and not args.no_gather_leg:
        leg("gather", gather_leg)

    def allreduce_leg():
        """SURVEY 8e's data-parallel fit of one shared mesh (tests/rasterise_tests.py:89): every rank renders its
        frames and the vertex gradient is summed over the frames and the ranks by one all-reduce per step
        (sharding.allreduce_shared_gradient, 16 V bytes).  Eager steps with and without the collective."""
        from dirt_amd.sharding import allreduce_shared_gradient
        n_s = max(20, args.steps // 2)

        def plain():
            step()

        def with_ar():
            step()
            allreduce_shared_gradient(sess.grad_vertices)

        for _ in range(3):
            with_ar()
        torch.cuda.synchronize()
        t_plain = timed(plain, n_s, barrier, world, device, shared)
        t_ar = timed(with_ar, n_s, barrier, world, device, shared)
        t_only = timed(lambda: allreduce_shared_gradient(sess.grad_vertices), n_s, barrier, world, device, shared)
        legs["shared_allreduce"] = {
            "what": "fwd+bwd per rank + one all-reduce of the shared vertex gradient [V,4] over %s per step "
                    "(eager steps)" % ("gloo (shared-GPU rehearsal)" if shared else "RCCL / xGMI"),
            "allreduce_bytes": V * 4 * 4,
            "allreduce_ms": round(t_only * 1e3 / n_s, 4),
            "value_eager_without": round(world * B * H * W * n_s / t_plain / 1e6, 1),
            "value_with_allreduce": round(world * B * H * W * n_s / t_ar / 1e6, 1),
            "ms_per_step_with_allreduce": round(t_ar * 1e3 / n_s, 4)}

    def batched_leg():
        """The same frames eight to a launch (config 3 x 8): the kernels at their steady state, without a single
        frame's launch ramp and drain (profiles/r05/pmc_bound/README.md) -- the rate the batched configuration
        C5 runs at.  Per-frame kernel times by HIP events and the backward's HBM fractions on them."""
        cfg8 = CONFIGS["c3x8"]
        B8 = cfg8[0]
        _, (bg8, v8, c8, f8), g8, _ = make_inputs(cfg8, rank, device)
        s8 = RasteriseSession(B8, H, W, C, V, F, device=device)

        def step8():
            s8.forward(bg8, v8, c8, f8)
            s8.backward(g8)

        for _ in range(3):
            step8()
        n8 = max(5, args.steps // 8)
        g_8 = graph_of(step8, n8, cap_stream) if not args.no_graph else None
        t8 = timed(g_8.replay if g_8 else lambda: [step8() for _ in range(n8)], 1, barrier, world, device, shared)
        k8 = kernel_times(step8, max(2, args.profile_steps // 8))
        per = {k: u / B8 for k, u in k8.items()}
        out8 = {"what": "%d config-3 frames per launch (seeds %d..), per-frame kernel times by HIP events" % (B8, rank * B8),
                "mpix_s": round(world * B8 * H * W * n8 / t8 / 1e6, 1),
                "kernels_us_per_frame": {k: round(u, 2) for k, u in per.items()},
                "grad_kernel_frac": round(kbytes["grad_kernel"] / (per["grad_kernel"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        if traffic is not None and dom == "grad_kernel":
            out8["grad_traffic_frac"] = round(traffic / (per["grad_kernel"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        legs["batched_steady_state"] = out8
        del g_8, s8

    def deep_leg():
        """The r = 64 px stress distribution (config 3's frame with large triangles, depth complexity ~45): the
        default forward, which picks the occluder-culling raster by itself (ABI 12), against the plain
        raster forced (DIRT_FWD_DEEP_CULL_OFF).  Graph-replayed fwd+bwd steps and the raster's event time."""
        cfgd = CONFIGS["c3_r64"]
        _, (bgd, vd, cd, fd), gd, _ = make_inputs(cfgd, rank, device)
        out = {"what": "config-3 frame of r = 64 px triangles: automatic deep culling vs the plain raster"}
        for name, dc in (("default", None), ("plain", False)):
            sd = RasteriseSession(B, H, W, C, V, F, device=device, deep_cull=dc)

            def stepd():
                sd.forward(bgd, vd, cd, fd)
                sd.backward(gd)

            for _ in range(4):
                stepd()
            torch.cuda.synchronize()
            nd = max(10, args.steps // 10)
            g_d = graph_of(stepd, nd, cap_stream) if not args.no_graph else None
            td = timed(g_d.replay if g_d else lambda: [stepd() for _ in range(nd)], 1, barrier, world, device, shared)
            kd = kernel_times(stepd, max(2, args.profile_steps // 4))
            out[name] = {"mpix_s": round(world * B * H * W * nd / td / 1e6, 1),
                         "kernels_us": {k: round(u, 2) for k, u in kd.items()}}
            del g_d, sd
        out["rule_state"] = _lib.deep_cull_state()
        legs["deep_scene"] = out

    # ---- leg: eight frames per launch, the kernels' steady state (config 3 only)
    if args.config == "c3" and args.rotate > 1:
        leg("batched_steady_state", batched_leg)

    # ---- leg (N > 1): the shared-parameter gradient all-reduce of a data-parallel pose fit
    if world > 1 and not args.no_gather_leg:
        leg("shared_allreduce", allreduce_leg)

    # ---- leg: a deep scene under the default forward (config 3's shape, r = 64 px; last: it leaves the device's
    # automatic deep-cull rule on for a few forwards)
    if args.config == "c3" and args.rotate > 1:
        leg("deep_scene", deep_leg)

    # R5 deviation counters over every forward the headline session ran: faces culled by the R5
    # vertex cap, clipped faces moved by the R5 sub-vertex clamp (0 expected on these scenes)
    try:
        clip_stats = sess.clip_stats()
    except Exception as e:  # noqa: BLE001 -- informative field only
        clip_stats = {"error": str(e)[:200]}

    cpu = par = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ref = cpu_baseline(host, grad_host, budget_s=args.cpu_budget)
        step()  # one more step so that the session buffers hold this frame's forward and backward
        torch.cuda.synchronize()
        par = parity(sess, ref)

    if rank == 0:
        out = {
            "metric": "Mpixels/s fwd+bwd @1024^2 50k-tri",
            "value": round(value, 1), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "clock_warm": clock_warm, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "%s: %d frame(s)/rank x %d random tris (r=%gpx), %dx%dx%d, fwd+bwd" %
                                   (args.config, B, F, _r, H, W, C),
                       "frames_per_rank": B, "height": H, "width": W, "channels": C, "faces": F, "vertices": V,
                       "parallelism": "frames sharded over %d rank(s); no collective in the step (the output "
                                      "gather is measured as its own leg, legs.gather)" % world,
                       "hip_graph": not args.no_graph, "steps_per_graph": gs},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity_vs_oracle": par,
            "r5_clip_stats": clip_stats,
            "kernels_us": {k: round(u, 2) for k, u in kern_us.items()},
            "legs": legs,
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
