"""Kernels of the public op's fwd+bwd step captured in a HIP graph (bench.py's api_autograd leg) next to the
session step's, for a rocprofv3 --kernel-trace --stats run: which launches the op path adds.

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python3 tools/api_graph_kernels.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
import dirt_amd  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

dev = torch.device("cuda", 0)
cfg = bench.CONFIGS["c3"]
host, (bg, v, c, f), grad, _ = bench.make_inputs(cfg, 0, dev)
B, H, W, C = bg.shape
bg_r, v_r, c_r = (t.clone().requires_grad_(True) for t in (bg, v, c))


def api_step():
    px = dirt_amd.rasterise_batch(bg_r, v_r, c_r, f)
    torch.autograd.grad(px, [bg_r, v_r, c_r], grad)


sess = RasteriseSession(B, H, W, C, v.shape[1], f.shape[1], device=dev)


def sess_step():
    sess.forward(bg, v, c, f)
    sess.backward(grad)


s = torch.cuda.Stream(dev)
for name, step, n in (("api", api_step, 100), ("session", sess_step, 1000)):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    g = bench.graph_of(step, 1, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print("%-8s graph step %.2f us (%d replays)" % (name, e0.elapsed_time(e1) * 1e3 / n, n))
