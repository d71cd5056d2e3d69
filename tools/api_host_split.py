#!/usr/bin/env python3
"""Host time of the public op's eager step, split (c3, one process, interleaved so that every part sees the same
host placement): the C ABI forward alone through ctypes (two kernel launches), the C++ autograd function's forward
without and with a graph to record, the backward through torch.autograd.grad, and torch's own floor (a one-node
backward of y = 2x).  Host time = wall time of the call without synchronisation (the GPU work is queued).

    python tools/api_host_split.py [--reps 300]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    args = ap.parse_args()
    import bench
    from dirt_amd import _lib, rasterise_ops
    ext = rasterise_ops._torch_ext()
    rasterise_ops.set_geometry_sharing(False)
    dev = torch.device("cuda", 0)
    B, H, W, C, F, r = bench.CONFIGS["c3"]
    _, (bg, v, c, f), grad, _ = bench.make_inputs(bench.CONFIGS["c3"], 0, dev)
    V = v.shape[1]
    bgr, vr, cr = (t.clone().requires_grad_(True) for t in (bg, v, c))
    lib = _lib.load()
    saved_b, scratch_b = _lib.workspace_sizes(B, H, W, C, V, F)
    saved = torch.empty(saved_b, dtype=torch.uint8, device=dev)
    scratch = torch.zeros(scratch_b, dtype=torch.uint8, device=dev)
    px = torch.empty((B, H, W, C), device=dev)
    gb = torch.empty((B, H, W), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    x = torch.ones(1024, device=dev, requires_grad=True)
    gx = torch.ones(1024, device=dev)
    out = {}

    def cabi_fwd():
        lib.dirt_rasterise_fwd(bg.data_ptr(), v.data_ptr(), c.data_ptr(), f.data_ptr(), None, B, H, W, C, V, F, 0,
                               px.data_ptr(), gb.data_ptr(), saved.data_ptr(), saved_b, scratch.data_ptr(),
                               scratch_b, 0, 0, None, None, stream)

    def fwd_nograd():
        with torch.no_grad():
            ext.rasterise_checked(bg, v, c, f, H, W, C, 0, False, False)

    def fwd_grad():
        out["px"] = ext.rasterise_checked(bgr, vr, cr, f, H, W, C, 0, False, False)[0]

    def bwd():
        torch.autograd.grad(out.pop("px"), [bgr, vr, cr], grad)

    def public_step():
        p = rasterise_ops._rasterise_batched(bgr, vr, cr, f, None, H, W, C, 0, 0)
        torch.autograd.grad(p, [bgr, vr, cr], grad)

    def engine_floor():
        torch.autograd.grad(x * 2.0, [x], gx)

    parts = {"cabi_fwd (2 launches, ctypes)": cabi_fwd, "ext fwd, no graph": fwd_nograd,
             "ext fwd, graph recorded": fwd_grad, "autograd.grad (op backward)": bwd,
             "public step (wrapper fwd + grad)": public_step, "engine floor (y = 2x backward)": engine_floor}
    times = {k: [] for k in parts}
    for _ in range(20):
        for k, fn in parts.items():
            if k.startswith("autograd.grad"):
                fwd_grad()
            fn()
    torch.cuda.synchronize()
    for _ in range(args.reps):
        for k, fn in parts.items():
            if k.startswith("autograd.grad"):
                fwd_grad()
                torch.cuda.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            times[k].append((time.perf_counter() - t0) * 1e6)
            torch.cuda.synchronize()
    for k, ts in times.items():
        print("%-36s host %7.2f us (median; p10 %.2f, p90 %.2f)" % (k, np.median(ts), np.percentile(ts, 10),
                                                                    np.percentile(ts, 90)))


if __name__ == "__main__":
    main()
