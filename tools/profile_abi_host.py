"""Host issue time of the C ABI calls themselves (ctypes, preallocated buffers, no autograd), against a torch
allocation and an empty kernel launch, at config 3.  Where the public op's backward host time goes beyond the
autograd engine (tools/profile_api_split.py).

    python tools/profile_abi_host.py
"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

dev = torch.device("cuda", 0)
cfg = bench.CONFIGS["c3"]
host, (bg, v, c, f), grad, _ = bench.make_inputs(cfg, 0, dev)
B, H, W, C = bg.shape
V, F = v.shape[1], f.shape[1]
sess = RasteriseSession(B, H, W, C, V, F, device=dev)
sess.forward(bg, v, c, f)
lib = _lib.load()
stream = torch.cuda.current_stream(dev).cuda_stream
gv = torch.empty((B, V, 4), device=dev)
gc = torch.empty((B, V, C), device=dev)
gbg = torch.empty((B, H, W, C), device=dev)
args_bwd = (v.data_ptr(), c.data_ptr(), f.data_ptr(), sess.pixels.data_ptr(), grad.data_ptr(),
            sess.gbuffer.data_ptr(), sess.saved.data_ptr(), B, H, W, C, V, F, gv.data_ptr(), gc.data_ptr(),
            gbg.data_ptr(), 0, stream)
x = torch.zeros(1, device=dev)
cases = {
    "abi_bwd (ctypes)": lambda: lib.dirt_rasterise_bwd(*args_bwd),
    "session.forward": lambda: sess.forward(bg, v, c, f),
    "session.backward": lambda: sess.backward(grad),
    "torch.empty 12.6 MB": lambda: torch.empty((B, H, W, C), device=dev),
    "torch add_ (1 launch)": lambda: x.add_(1.0),
    "ctypes abi_version": lambda: lib.dirt_abi_version(),
}
for name, fn in cases.items():
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    n = 300
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    print("%-24s host issue %7.2f us/call" % (name, t_host * 1e6))
