"""Throughput of every BASELINE.json config on one GPU ("report all"): forward+backward steps
through RasteriseSession replayed from HIP graphs (10 steps per graph), inputs resident in HBM; beside
each, the CPU oracle (test infrastructure, OpenMP on the job's host-core share) on the same frames
(BASELINE.md section 2's CPU column), and for c4 the whole deferred-shading chain of samples/deferred.py
(tests/deferred_pipeline.py) through the public op + autograd.

    python tools/bench_configs.py > profiles/r01/configs.jsonl
    python tools/bench_configs.py stress c5   # only the configs whose names contain these
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

CONFIGS = {
    "c1_readme_square_128x128x1": lambda: [scenes.readme_square()],
    "c2_cube_256x256x3": lambda: [scenes.cube_scene()],
    # the cube at 4096^2: 12 faces over 65536 tiles (past kFusedMaxTiles: setup launch + bins, not the fused
    # forward -- ADVICE r3's large-frame case)
    "c2_cube_4096x4096x3": lambda: [scenes.cube_scene(W=4096, H=4096)],
    "c3_random50k_1024x1024x3": lambda: [scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)],
    # config 3 frames eight to a launch: the kernels' steady-state time per frame (many workgroup rounds per CU,
    # so no first-round burst or drain tail in the per-frame figure)
    "c3x8_random50k_1024x1024x3_batch8": lambda: [scenes.random_triangles(F=50000, W=1024, H=1024, seed=b)
                                                  for b in range(8)],
    "c4_deferred20k_512x512x7": lambda: [scenes.deferred_mesh_scene()],
    # a quarter-size config-3 frame (one round of backward workgroups): the small-frame shape of the deferred renders
    "c3q_random20k_512x512x3": lambda: [scenes.random_triangles(F=20000, W=512, H=512, seed=0)],
    "c3q_mesh20k_512x512x3": lambda: [tuple(a[..., :3] if k in (0, 2) else a for k, a in enumerate(scenes.deferred_mesh_scene()))],
    "c5_batch8x20k_1024x1024x3_per_gpu": lambda: [scenes.random_triangles(F=20000, W=1024, H=1024, seed=b)
                                                  for b in range(8)],
    "c3_stress_r64_1024x1024x3": lambda: [scenes.random_triangles(F=50000, W=1024, H=1024, radius_px=64.0, seed=0)],
    # the same with the forward's occluder culling (DIRT_FWD_DEEP_CULL, RasteriseSession(deep_cull=True))
    "c3_stress_r64_1024x1024x3_deep_cull": lambda: [scenes.random_triangles(F=50000, W=1024, H=1024, radius_px=64.0,
                                                                            seed=0)],
    # a mesh crowded into the centre 1/16 of each frame at config 5's per-rank batch, at the
    # default bin capacity and with the slabs forced small (1024 entries: the crowded tiles overflow and take
    # the all-records path), to price the overflow path
    "c5_clustered_8x20k_centre16th": lambda: [scenes.random_triangles(F=20000, W=1024, H=1024, seed=200 + b,
                                                                      spread=0.25) for b in range(8)],
    "c5_clustered_8x20k_centre16th_slab1024": lambda: [scenes.random_triangles(F=20000, W=1024, H=1024,
                                                                               seed=200 + b, spread=0.25)
                                                       for b in range(8)],
}
# per-config bin capacity (entries in all slabs; 0 = default)
BIN_CAPACITY = {"c5_clustered_8x20k_centre16th_slab1024": 8 * 256 * 1024}


def bin_occupancy(B, H, W, F, cap, scratch, nbytes):
    import ctypes
    lib = _lib.load()
    fn = lib.dirt_debug_bin_occupancy
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p] + \
        [ctypes.POINTER(ctypes.c_uint32)] * 3
    mx, ov, slab = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(fn(B, H, W, F, cap, scratch.data_ptr(), nbytes, torch.cuda.current_stream().cuda_stream,
                  ctypes.byref(mx), ctypes.byref(ov), ctypes.byref(slab)))
    return {"max_slab_entries": mx.value, "overflowed_slabs": ov.value, "slab_capacity": slab.value}


def cpu_oracle(host, g, budget_s=3.0):
    """The CPU oracle's fwd+bwd on the same frames (median over repetitions within ~budget_s)."""
    from oracle import oracle
    import bench
    n = bench.cpu_threads()
    bg, v, c, f = host
    ts = []
    t_start = time.perf_counter()
    while not ts or (time.perf_counter() - t_start < budget_s and len(ts) < 20):
        t0 = time.perf_counter()
        px, gb, _ = oracle.rasterise_fwd(bg, v, c, f, nthreads=n)
        oracle.rasterise_bwd(v, c, f, px, g, gb, nthreads=n)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    return {"cpu_Mpixels_per_s": round(bg.shape[0] * bg.shape[1] * bg.shape[2] / t / 1e6, 2), "cpu_threads": n,
            "cpu_ms_per_step": round(t * 1e3, 2)}


def deferred_chain(steps=20, batched=False):
    """c4 as the reference sample runs it: three 3-channel G-buffer renders + dilation + lighting + loss,
    backward to world-space vertices (tests/deferred_pipeline.py), through dirt_amd.rasterise + autograd.
    Reported eager (host-issued every step), as one captured HIP graph per step (device time: the whole
    chain replayed, no host work), and the host's issue time alone (eager wall time minus nothing queued)."""
    import deferred_pipeline as dp
    dev = torch.device("cuda", 0)
    H = W = 512
    world, faces, albedo = dp.grid_surface()
    Vw = torch.from_numpy(world).to(dev).requires_grad_(True)
    f = torch.from_numpy(faces).to(dev)
    al = torch.from_numpy(albedo).to(dev)
    wts = torch.rand((H, W, 3), device=dev)
    out = {}

    def step():
        L, _, _ = dp.chain(dp.hip_render, Vw, f, al, H, W, wts, batched=batched)
        out["g"] = torch.autograd.grad(L, [Vw])[0]

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ref = out["g"].clone()
    # host issue time: the same steps with the device already busy is what eager costs; time the Python /
    # autograd work alone by issuing without synchronising and reading the host clock
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t_issue = (time.perf_counter() - t0) / steps
    torch.cuda.synchronize()
    res = {"config": "c4_deferred_chain_3x512x512x3_grad_to_world_vertices" + ("_batched" if batched else ""),
           "faces": len(faces),
           "ms_per_step_eager": round(dt * 1e3, 3), "host_issue_ms_per_step": round(t_issue * 1e3, 3),
           "Mpixels_per_s_fwd_bwd": round(H * W / dt / 1e6, 1)}
    try:
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            step()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        dg = e0.elapsed_time(e1) / steps
        err = float((out["g"] - ref).abs().max() / ref.abs().max())
        res.update({"ms_per_step_graph": round(dg, 4), "Mpixels_per_s_graph": round(H * W / (dg * 1e-3) / 1e6, 1),
                    "graph_grad_rel_diff_vs_eager": err})
        del graph
    except Exception as e:  # noqa: BLE001 -- reported, not fatal
        res["graph_error"] = "%s: %s" % (type(e).__name__, str(e)[:200])
    return res


def run(name, frames, steps=100):
    host = [np.stack([fr[k] for fr in frames]) for k in range(4)]
    dev = torch.device("cuda", 0)
    bg, v, c, f = (torch.from_numpy(a).to(dev) for a in host)
    B, H, W, C = bg.shape
    V, F = v.shape[1], f.shape[1]
    g = torch.randn((B, H, W, C), device=dev)
    cap = BIN_CAPACITY.get(name, 0)
    sess = RasteriseSession(B, H, W, C, V, F, device=dev, bin_capacity=cap, deep_cull=True if name.endswith("deep_cull") else None)

    def step():
        sess.forward(bg, v, c, f)
        sess.backward(g)

    for _ in range(5):
        step()
    sess.forward(bg, v, c, f)
    occ = bin_occupancy(B, H, W, F, cap, sess.scratch, sess.scratch_bytes)
    sess.backward(g)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(10):
            step()
    graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // 10):
        graph.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (steps // 10 * 10)
    _lib.profile_enable(True)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.profile_enable(False)
    out = {"config": name, "frames": B, "H": H, "W": W, "C": C, "faces": F, "vertices": V,
           "Mpixels_per_s_fwd_bwd": round(B * H * W / dt / 1e6, 1), "us_per_step": round(dt * 1e6, 2),
           "kernels_us": {k: round(ms / n * 1e3, 2) for k, (n, ms) in prof.items() if n}, "bins": occ}
    if os.environ.get("DIRT_NO_CPU") != "1":
        out.update(cpu_oracle(host, g.cpu().numpy()))
        out["gpu_over_cpu"] = round(out["Mpixels_per_s_fwd_bwd"] / max(out["cpu_Mpixels_per_s"], 1e-9), 1)
    return out


def main():
    # optional arguments: substrings selecting configs (all by default)
    sel = sys.argv[1:]
    for name, make in CONFIGS.items():
        if not sel or any(k in name for k in sel):
            print(json.dumps(run(name, make())), flush=True)
    if not sel or any(k in "c4_deferred_chain" for k in sel):
        print(json.dumps(deferred_chain()), flush=True)
        print(json.dumps(deferred_chain(batched=True)), flush=True)


if __name__ == "__main__":
    main()
