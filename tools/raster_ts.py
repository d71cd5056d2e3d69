"""Per-phase timestamps of the instrumented forward raster (raster_kernel<3,128>) at config 3.

Wave 0 of every workgroup records s_memtime at: start (0), bin filter done (1, first chunk barrier),
first staging round done (2), entry loop done (3), resolve loads landed (4: the own record and FaceData,
lambda computed), outputs issued (5).  Prints median / mean phase durations, the workgroup lifetime and
the mean number of workgroups resident per CU."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

PH = ["bin filter", "staging", "entry loop (wave 0)", "resolve loads", "resolve + stores"]


def main():
    dev = torch.device("cuda", 0)
    bg, v, c, f = scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)
    t = [torch.from_numpy(a[None]).to(dev) for a in (bg, v, c, f)]
    B, H, W, C = t[0].shape
    V, F = t[1].shape[1], t[3].shape[1]
    sess = RasteriseSession(B, H, W, C, V, F, device=dev)
    sess.forward(*t)
    lib = _lib.load()
    P = ctypes.c_void_p
    rfn = lib.dirt_debug_raster_variant
    rfn.argtypes = [ctypes.c_int, P, P, P, P] + [ctypes.c_int] * 6 + [P, P, P, P, P, ctypes.POINTER(ctypes.c_float)]
    rfn.restype = ctypes.c_int
    rd = lib.dirt_debug_read_phase_ts
    rd.argtypes = [P, ctypes.c_int]
    stream = torch.cuda.current_stream().cuda_stream
    ms = ctypes.c_float(0)
    nwg = ((W + 15) // 16) * ((H + 15) // 16) * B  # raster tiles are 16 x 16
    for variant in (0, 128, 0, 128):
        _lib.check(rfn(variant, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), B, H, W, C, V, F,
                       sess.pixels.data_ptr(), sess.gbuffer.data_ptr(), sess.saved.data_ptr(), sess.scratch.data_ptr(),
                       stream, ctypes.byref(ms)))
        print("variant %d: %.2f us" % (variant, ms.value * 1e3))
    ts = np.zeros((nwg, 13), np.uint64)
    _lib.check(rd(ts.ctypes.data, nwg))
    T = ts[:, :6].astype(np.int64)
    hw = ts[:, 8].astype(np.int64)
    xcc = ts[:, 9].astype(np.int64) & 0xf
    cu = (hw >> 8) & 0xf
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    spans, resident = [], []
    for x in np.unique(key):
        m = key == x
        T[m] -= T[m, 0].min()
        spans.append(T[m, 5].max())
        resident.append((T[m, 5] - T[m, 0]).sum() / max(T[m, 5].max(), 1))
    span = float(np.median(spans))
    tick_us = ms.value * 1e3 / span
    print("per-CU span median %.0f ticks ~ kernel %.2f us -> %.2f MHz; %d CUs, %.1f workgroups resident per CU" % (
        span, ms.value * 1e3, 1.0 / tick_us, len(spans), float(np.mean(resident))))
    d = np.diff(T, axis=1)
    for k, name in enumerate(PH):
        print("  %-22s median %8.0f  p90 %8.0f  mean %8.0f ticks  (%.2f us)" % (
            name, np.median(d[:, k]), np.percentile(d[:, k], 90), d[:, k].mean(), d[:, k].mean() * tick_us))
    life = T[:, 5] - T[:, 0]
    print("  %-22s median %8.0f  p90 %8.0f  mean %8.0f ticks  (%.2f us)" % (
        "workgroup life", np.median(life), np.percentile(life, 90), life.mean(), life.mean() * tick_us))
    # dispatch: workgroups per CU and how late they started (rebased per CU)
    cnt = np.bincount(key)
    cnt = cnt[cnt > 0]
    late = T[:, 0] > 0.25 * span
    print("  WGs per CU: min %d median %d max %d; started after 25%% of the span: %d of %d" % (
        cnt.min(), np.median(cnt), cnt.max(), late.sum(), len(late)))
    for q in (10, 50, 90, 99):
        print("  start p%d %.2f us, end p%d %.2f us" % (q, np.percentile(T[:, 0], q) * tick_us, q,
                                                    np.percentile(T[:, 5], q) * tick_us))


if __name__ == "__main__":
    main()
