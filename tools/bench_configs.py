"""Throughput of every BASELINE.json config on one GPU ("report all"): forward+backward steps
through RasteriseSession replayed from HIP graphs (10 steps per graph), inputs resident in HBM.

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
    "c3_random50k_1024x1024x3": lambda: [scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)],
    "c4_deferred20k_512x512x7": lambda: [scenes.deferred_mesh_scene()],
    "c5_batch8x20k_1024x1024x3_per_gpu": lambda: [scenes.random_triangles(F=20000, W=1024, H=1024, seed=b)
                                                  for b in range(8)],
    "c3_stress_r64_1024x1024x3": lambda: [scenes.random_triangles(F=50000, W=1024, H=1024, radius_px=64.0, seed=0)],
}


def run(name, frames, steps=100):
    host = [np.stack([fr[k] for fr in frames]) for k in range(4)]
    dev = torch.device("cuda", 0)
    bg, v, c, f = (torch.from_numpy(a).to(dev) for a in host)
    B, H, W, C = bg.shape
    V, F = v.shape[1], f.shape[1]
    g = torch.randn((B, H, W, C), device=dev)
    sess = RasteriseSession(B, H, W, C, V, F, device=dev)

    def step():
        sess.forward(bg, v, c, f)
        sess.backward(g)

    for _ in range(5):
        step()
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
    return {"config": name, "frames": B, "H": H, "W": W, "C": C, "faces": F, "vertices": V,
            "Mpixels_per_s_fwd_bwd": round(B * H * W / dt / 1e6, 1), "us_per_step": round(dt * 1e6, 2),
            "kernels_us": {k: round(ms / n * 1e3, 2) for k, (n, ms) in prof.items() if n}}


def main():
    # optional arguments: substrings selecting configs (all by default)
    sel = sys.argv[1:]
    for name, make in CONFIGS.items():
        if not sel or any(k in name for k in sel):
            print(json.dumps(run(name, make())), flush=True)


if __name__ == "__main__":
    main()
