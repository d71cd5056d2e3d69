"""Probe: the backward's grad_background stores -- the grad launch timed by HIP events with grad_background written
(the session's backward) and with it NULL (dirt_rasterise_bwd skips those stores), config 3, interleaved."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    _, (bg, v, c, f), g, _ = bench.make_inputs(bench.CONFIGS["c3"], 0, dev)
    B, H, W, C = bg.shape
    V, F = v.shape[1], f.shape[1]
    s = RasteriseSession(B, H, W, C, V, F, device=dev)
    s.forward(bg, v, c, f)
    s.backward(g)
    lib = _lib.load()
    stream = torch.cuda.current_stream().cuda_stream
    gv = torch.empty((B, V, 4), device=dev)
    gc = torch.empty((B, V, C), device=dev)
    gbg = torch.empty((B, H, W, C), device=dev)

    def bwd(with_bg):
        _lib.check(lib.dirt_rasterise_bwd(v.data_ptr(), c.data_ptr(), f.data_ptr(), s.pixels.data_ptr(), g.data_ptr(),
                                          s.gbuffer.data_ptr(), s.saved.data_ptr(), B, H, W, C, V, F, gv.data_ptr(),
                                          gc.data_ptr(), gbg.data_ptr() if with_bg else None, 0, stream))

    out = {}
    for r in range(3):
        for wb in (True, False):
            for _ in range(5):
                bwd(wb)
            _lib.profile_enable(True)
            for _ in range(50):
                bwd(wb)
            torch.cuda.synchronize()
            prof = _lib.profile_read()
            _lib.profile_enable(False)
            n, ms = prof["grad_kernel"]
            out.setdefault("with_grad_bg" if wb else "without_grad_bg", []).append(round(ms / n * 1e3, 2))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
