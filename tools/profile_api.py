"""Host-side cost of the public op path (dirt_amd.rasterise_batch + torch.autograd.grad), c3 frame:
wall time per eager step, and a cProfile of the Python side (where the non-GPU time goes)."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
import dirt_amd  # noqa: E402

dev = torch.device("cuda", 0)
cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
host, (bg, v, c, f), grad, _ = bench.make_inputs(cfg, 0, dev)
t = [x.clone().requires_grad_(True) for x in (bg, v, c)]


def step():
    px = dirt_amd.rasterise_batch(t[0], t[1], t[2], f)
    torch.autograd.grad(px, t, grad)


for _ in range(20):
    step()
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for _ in range(n):
    step()
torch.cuda.synchronize()
print("eager step %.1f us" % ((time.perf_counter() - t0) / n * 1e6))
# host-only time: the same calls, timed without waiting for the GPU (queue runs ahead)
t0 = time.perf_counter()
for _ in range(50):
    step()
t_host = (time.perf_counter() - t0) / 50
torch.cuda.synchronize()
print("host issue time per step %.1f us" % (t_host * 1e6))
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
