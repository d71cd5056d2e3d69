"""Where the public op's host time goes (c3 frame): host issue time per call of each layer, the GPU queue
running ahead (no synchronisation inside the timed loops).

  fwd_nograd_ext   _dirt_torch.rasterise without autograd (allocation + ABI + 2 launches)
  fwd_grad_ext     the same with inputs requiring grad (autograd node, saved tensors, accumulator zero-fill)
  fwd_grad_py      dirt_amd.rasterise_batch (Python argument handling on top)
  fwd_bwd_ext      _dirt_torch.rasterise + torch.autograd.grad
  fwd_bwd_py       dirt_amd.rasterise_batch + torch.autograd.grad (the bench's api leg)
  bwd_only         torch.autograd.grad on a graph built outside the timed loop (retain_graph)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
import dirt_amd  # noqa: E402
from dirt_amd import rasterise_ops  # noqa: E402

dev = torch.device("cuda", 0)
cfg = bench.CONFIGS["c3"]
host, (bg, v, c, f), grad, _ = bench.make_inputs(cfg, 0, dev)
t = [x.clone().requires_grad_(True) for x in (bg, v, c)]
ext = rasterise_ops._torch_ext()
B, H, W, C = bg.shape


def ext_call(a, b, cc):
    return ext.rasterise(a, b, cc, f, None, H, W, C, 0, 0, False, False)[0]


cases = {
    "fwd_nograd_ext": lambda: ext_call(bg, v, c),
    "fwd_grad_ext": lambda: ext_call(*t),
    "fwd_grad_py": lambda: dirt_amd.rasterise_batch(t[0], t[1], t[2], f),
    "fwd_bwd_ext": lambda: torch.autograd.grad(ext_call(*t), t, grad),
    "fwd_bwd_py": lambda: torch.autograd.grad(dirt_amd.rasterise_batch(t[0], t[1], t[2], f), t, grad),
}
if "graph" in sys.argv[1:]:
    # as bench.py does before its api leg: a session's 200-step HIP graph captured and replayed first
    from dirt_amd.session import RasteriseSession
    sess = RasteriseSession(B, H, W, C, v.shape[1], f.shape[1], device=dev)

    def sstep():
        sess.forward(bg, v, c, f)
        sess.backward(grad)

    for _ in range(5):
        sstep()
    g = bench.graph_of(sstep, 200, torch.cuda.Stream(dev))
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print("(after a 200-step session graph)")
px_keep = ext_call(*t)
cases["bwd_only"] = lambda: torch.autograd.grad(px_keep, t, grad, retain_graph=True)
# the autograd engine's own cost for a one-node CUDA graph (torch's mul backward), for comparison
xm = torch.randn(B, H, W, C, device=dev, requires_grad=True)
ym = xm * 2.0
cases["engine_mul_bwd"] = lambda: torch.autograd.grad(ym, xm, grad, retain_graph=True)
for name, fn in cases.items():
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / n
    print("%-16s host issue %7.1f us/call   wall incl. GPU %7.1f us/call" % (name, t_host * 1e6, t_all * 1e6))
