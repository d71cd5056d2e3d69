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
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r02", "traffic.json")

CONFIGS = {
    # name: (B per rank, H, W, C, F, radius_px)
    "c3": (1, 1024, 1024, 3, 50000, 16.0),
    "c5": (8, 1024, 1024, 3, 20000, 16.0),  # 64 frames over 8 GPUs -> 8 per rank
    "c3_r64": (1, 1024, 1024, 3, 50000, 64.0),
}


def alg_bytes(B, H, W, C, V, F):
    """Algorithmic HBM bytes (tensor I/O of the op) per kernel and per op."""
    hwc, hw = 4 * C * H * W, 4 * H * W
    k = {
        "raster_kernel": B * (2 * hwc + hw + 4 * C * V + 12 * F),
        "grad_kernel": B * (3 * hwc + hw + 16 * V + 12 * F + 16 * V + 4 * C * V),
        "setup_kernel": B * (12 * F + 16 * V),
    }
    fwd = B * (16 * V + 12 * F + 4 * C * V + 2 * hwc)
    bwd = B * (16 * V + 12 * F + 4 * C * V + 2 * hwc + 16 * V + 4 * C * V + hwc)
    return k, fwd, bwd


def make_inputs(cfg, rank, device):
    import scenes
    B, H, W, C, F, r = cfg
    frames = [scenes.random_triangles(F=F, W=W, H=H, C=C, radius_px=r, seed=rank * B + b) for b in range(B)]
    host = [np.stack([fr[k] for fr in frames]) for k in range(4)]
    dev = [torch.from_numpy(a).to(device) for a in host]
    g = np.random.default_rng(10_000 + rank).standard_normal(host[0].shape).astype(np.float32)
    return host, dev, torch.from_numpy(g).to(device), g


def cpu_baseline(host, grad_host, budget_s=10.0, max_reps=20):
    from oracle import oracle
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
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
    return {"value": B * H * W / t / 1e6, "unit": "Mpixels/s", "cores": nthreads, "kind": "port",
            "sample": "%d x full config frame(s) (%dx%dx%d, F=%d) fwd+bwd, median of %d reps, oracle/dirt_oracle.c "
                      "OpenMP" % (B, H, W, C, f.shape[1], len(times)),
            "ms_per_frame": t * 1e3 / B}, (px, gb) + tuple(grads)


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
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # DIRT_BENCH_SHARED_GPU=1: rehearsal of the N-rank path on a box with fewer GPUs than ranks (ranks share
    # cuda:LOCAL_RANK % count, timing reduced over gloo); the driver's multi-GPU runs leave it unset (RCCL)
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

    def step():
        sess.forward(bg, v, c, f)
        sess.backward(grad)

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    # the timed loop runs exactly args.steps complete steps: full graph replays of gs steps each, the
    # remainder eagerly
    gs = 1 if args.no_graph else max(1, min(args.graph_steps, args.steps))
    n_replays, n_rest = divmod(args.steps, gs)
    run = step
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(gs):
                step()
        for _ in range(2):
            graph.replay()
        run = graph.replay
    else:
        n_replays, n_rest = args.steps, 0

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_replays):
        run()
    for _ in range(n_rest):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * B * H * W * args.steps / elapsed / 1e6

    # per-kernel HIP-event timing (same kernels, eager launches, outside the timed loop)
    _lib.profile_enable(True)
    for _ in range(args.profile_steps):
        step()
    torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.profile_enable(False)
    kern_us = {k: (ms / n * 1e3 if n else 0.0) for k, (n, ms) in prof.items()}
    kbytes, fwd_b, bwd_b = alg_bytes(B, H, W, C, V, F)
    dom = max((k for k in kern_us if k in kbytes), key=lambda k: kern_us[k])
    achieved = kbytes[dom] / (kern_us[dom] * 1e-6) / 1e9
    traffic = None
    if args.config == "c3" and os.path.exists(TRAFFIC_JSON):
        tk = json.load(open(TRAFFIC_JSON)).get("kernels", {})
        hit = [v for k, v in tk.items() if k.split("<")[0] == dom]
        if hit:
            traffic = hit[0]["traffic_bytes"]
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": os.path.relpath(TRAFFIC_JSON, ROOT) if traffic is not None else None,
                "alg_bytes_per_launch": kbytes[dom], "avg_us": round(kern_us[dom], 2),
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
        roofline["traffic_frac"] = round(traffic / (kern_us[dom] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)

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
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "%s: %d frame(s)/rank x %d random tris (r=%gpx), %dx%dx%d, fwd+bwd" %
                                   (args.config, B, F, _r, H, W, C),
                       "frames_per_rank": B, "height": H, "width": W, "channels": C, "faces": F, "vertices": V,
                       "parallelism": "frames sharded over %d rank(s), no collective in step" % world,
                       "hip_graph": not args.no_graph, "steps_per_graph": gs},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity_vs_oracle": par,
            "kernels_us": {k: round(u, 2) for k, u in kern_us.items()},
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
