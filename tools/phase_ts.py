"""Per-phase timestamps of the instrumented backward (grad_kernel<3,128>) at config 3 (`c4` argument: config 4).

Prints the median / p90 duration of each phase per workgroup, the workgroup lifetime, and how many
workgroups were resident per CU on average (from HW_ID / XCC_ID)."""
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

PH = ["load gb/G/I", "scalars+own inserts", "ring inserts", "slot record loads", "phase B (pairs)",
      "DPP+tails", "flush"]


def main():
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1 and sys.argv[1] == "c4":  # config 4: shared-vertex mesh, 512^2 x 7 (grad_kernel<7,128>)
        bg, v, c, f = scenes.deferred_mesh_scene()
    else:
        bg, v, c, f = scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)
    t = [torch.from_numpy(a[None]).to(dev) for a in (bg, v, c, f)]
    B, H, W, C = t[0].shape
    V, F = t[1].shape[1], t[3].shape[1]
    sess = RasteriseSession(B, H, W, C, V, F, device=dev)
    sess.forward(*t)
    g = torch.randn_like(sess.pixels)
    lib = _lib.load()
    fn = lib.dirt_debug_bwd_variant
    P = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, P, P, P, P] + [ctypes.c_int] * 6 + [P, P, P, P, ctypes.POINTER(ctypes.c_float)]
    rd = lib.dirt_debug_read_phase_ts
    rd.argtypes = [P, ctypes.c_int]
    stream = torch.cuda.current_stream().cuda_stream
    ms = ctypes.c_float(0)
    nwg = ((W + 15) // 16) * ((H + 15) // 16) * B
    for variant in (0, 128, 128, 128):
        _lib.check(fn(variant, sess.pixels.data_ptr(), g.data_ptr(), sess.gbuffer.data_ptr(), sess.saved.data_ptr(),
                      B, H, W, C, V, F, sess.grad_vertices.data_ptr(), sess.grad_vertex_colors.data_ptr(),
                      sess.grad_background.data_ptr(), stream, ctypes.byref(ms)))
        print("variant %d: %.2f us" % (variant, ms.value * 1e3))
    ts = np.zeros((nwg, 13), np.uint64)
    _lib.check(rd(ts.ctypes.data, nwg))
    T = ts[:, :8].astype(np.int64)
    hw = ts[:, 8].astype(np.int64)
    xcc = ts[:, 9].astype(np.int64) & 0xf
    cu = (hw >> 8) & 0xf
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    # s_memtime counters are not synchronised across CUs: rebase each CU on its first workgroup start
    spans = []
    for x in np.unique(key):
        m = key == x
        T[m] -= T[m, 0].min()
        spans.append(T[m, 7].max())
    span = float(np.median(spans))
    tick_us = ms.value * 1e3 / span
    print("per-CU span median %.0f ticks (min %d max %d) ~ kernel %.2f us -> %.2f MHz" % (
        span, min(spans), max(spans), ms.value * 1e3, 1.0 / tick_us))
    d = np.diff(T, axis=1)
    for k, name in enumerate(PH):
        print("  %-22s median %8.0f  p90 %8.0f  mean %8.0f ticks  (%.2f us)" % (
            name, np.median(d[:, k]), np.percentile(d[:, k], 90), d[:, k].mean(), d[:, k].mean() * tick_us))
    S = ts[:, 10:13].astype(np.int64)
    ok = (S[:, 0] > 0) & (S[:, 1] > 0)
    base = ts[:, 0].astype(np.int64)
    for k, name in enumerate(["B: own record", "B: pass 1 (ownership)", "B: pass 2 + colour + DPP"]):
        a = (ts[ok, 3 + k + (1 if k == 0 else 0) if False else 0]).astype(np.int64)
    b0 = ts[ok, 4].astype(np.int64)
    s10, s11, b5 = S[ok, 0], S[ok, 1], ts[ok, 5].astype(np.int64)
    for name, x in (("B: own record", s10 - b0), ("B: pass 1 (ownership)", s11 - s10), ("B: pass 2..barrier", b5 - s11)):
        print("  %-22s median %8.0f  p90 %8.0f  mean %8.0f ticks  (%.2f us)  [%d WGs]" % (
            name, np.median(x), np.percentile(x, 90), x.mean(), x.mean() * tick_us, ok.sum()))
    x = ts[:, 12].astype(np.int64) - ts[:, 1].astype(np.int64)
    print("  %-22s median %8.0f  mean %8.0f ticks  (%.2f us)" % ("A: pair scalars", np.median(x), x.mean(), x.mean() * tick_us))
    life = T[:, 7] - T[:, 0]
    print("  lifetime               median %8.0f  p90 %8.0f ticks  (%.2f us)" % (np.median(life), np.percentile(life, 90),
                                                                            life.mean() * tick_us))
    cnt = np.bincount(key)
    cnt = cnt[cnt > 0]
    print("  distinct CUs %d; WGs per CU: min %d max %d" % (len(cnt), cnt.min(), cnt.max()))
    # resident workgroups per CU over time (1% steps of the span)
    grid = np.linspace(0, span, 101)
    res = np.zeros((len(np.unique(key)), 101))
    for n, kk in enumerate(np.unique(key)):
        m = key == kk
        s0, s1 = T[m, 0], T[m, 7]
        res[n] = ((s0[None, :] <= grid[:, None]) & (s1[None, :] > grid[:, None])).sum(1)
    prof = res.mean(0)
    print("  mean resident WGs per CU over the span (10%% steps): " + " ".join("%.1f" % prof[k] for k in range(0, 101, 10)))
    print("  time-average resident %.2f, max %d" % (prof.mean(), res.max()))
    firsts = np.array([T[key == kk, 0].min() for kk in np.unique(key)])
    lasts = np.array([T[key == kk, 7].max() for kk in np.unique(key)])
    print("  per-CU first start median %.0f, last end median %.0f ticks" % (np.median(firsts), np.median(lasts)))


if __name__ == "__main__":
    main()
