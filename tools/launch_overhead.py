"""Fixed cost of a timed window: wall time of K bench steps (c3) as one HIP graph replay, as K eager steps,
and as K one-step graph replays, for several K; fits wall = a + b K.  The driver times bench.py with a
small K (20), so the fixed cost a is part of its number."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

dev = torch.device("cuda", 0)
cfg = bench.CONFIGS["c3"]
B, H, W, C, F, _ = cfg
host, (bg, v, c, f), grad, _ = bench.make_inputs(cfg, 0, dev)
sess = RasteriseSession(B, H, W, C, 3 * F, F, device=dev)


def step():
    sess.forward(bg, v, c, f)
    sess.backward(grad)


for _ in range(10):
    step()
torch.cuda.synchronize()
s = torch.cuda.Stream()
res = {}
for K in (1, 2, 5, 10, 20, 50, 100, 200):
    g = bench.graph_of(step, K, s)
    walls = []
    for rep in range(7):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    res[("graph", K)] = float(np.median(walls))
    del g
g1 = bench.graph_of(step, 1, s)
for K in (1, 5, 20, 50):
    for mode in ("eager", "graph1"):
        walls = []
        for rep in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                (step if mode == "eager" else g1.replay)()
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
        res[(mode, K)] = float(np.median(walls))
for mode in ("graph", "eager", "graph1"):
    ks = sorted(k for m, k in res if m == mode)
    w = np.array([res[(mode, k)] for k in ks]) * 1e6
    b_, a_ = np.polyfit(ks, w, 1)
    print("%-7s " % mode + "  ".join("K=%d %.0f us" % (k, x) for k, x in zip(ks, w)) +
          "   fit: %.1f us + %.2f us/step" % (a_, b_))

# the same K-step graph launched three ways: torch's replay(); after hipGraphUpload (the executable graph's
# device-side resources set up ahead of the timed window); hipGraphLaunch through ctypes (no torch wrapper)
import ctypes  # noqa: E402

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for K in (20, 200):
    g = bench.graph_of(step, K, s)
    ex = ctypes.c_void_p(g.raw_cuda_graph_exec())
    st = ctypes.c_void_p(s.cuda_stream)
    out = []
    for mode in ("replay", "upload+replay", "ctypes launch"):
        walls = []
        for rep in range(7):
            if mode == "upload+replay":
                assert hip.hipGraphUpload(ex, st) == 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "ctypes launch":
                assert hip.hipGraphLaunch(ex, st) == 0
            else:
                g.replay()
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
        out.append("%s %.0f us" % (mode, float(np.median(walls)) * 1e6))
    print("K=%d: " % K + ", ".join(out))
