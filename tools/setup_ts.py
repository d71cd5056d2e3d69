"""Per-phase timestamps of the instrumented setup kernel (setup_kernel<128>) at config 3.

Phases per workgroup: record setup (faces + vertices loads, R1-R5, record stores), LDS count flush,
slab reservation (returning device atomics), placement (LDS cursors + bin stores, drained)."""
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


def main():
    dev = torch.device("cuda", 0)
    bg, v, c, f = scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)
    t = [torch.from_numpy(a[None]).to(dev) for a in (bg, v, c, f)]
    B, H, W, C = t[0].shape
    V, F = t[1].shape[1], t[3].shape[1]
    sess = RasteriseSession(B, H, W, C, V, F, device=dev)
    lib = _lib.load()
    fn = lib.dirt_debug_setup_ts
    P = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, P, P] + [ctypes.c_int] * 5 + [P, P, P, ctypes.POINTER(ctypes.c_float)]
    rd = lib.dirt_debug_read_phase_ts
    rd.argtypes = [P, ctypes.c_int]
    stream = torch.cuda.current_stream().cuda_stream
    ms = ctypes.c_float(0)
    nwg = (F + 255) // 256 * B
    for variant, name in ((2, "plain"), (3, "plain, no reservation atomics"), (1, "timestamps, no reservation"),
                          (4, "no record arithmetic (bbox only)"), (5, "no record arithmetic, no reservation"),
                          (6, "reservation over two counters per tile")):
        tv = []
        for _ in range(20):
            _lib.check(fn(variant, t[1].data_ptr(), t[3].data_ptr(), B, H, W, V, F, sess.saved.data_ptr(),
                          sess.scratch.data_ptr(), stream, ctypes.byref(ms)))
            tv.append(ms.value * 1e3)
        print("setup variant %-32s median %.2f us" % (name, float(np.median(tv))))
    times = []
    for _ in range(5):
        _lib.check(fn(0, t[1].data_ptr(), t[3].data_ptr(), B, H, W, V, F, sess.saved.data_ptr(), sess.scratch.data_ptr(),
                      stream, ctypes.byref(ms)))
        times.append(ms.value * 1e3)
    print("setup_kernel<128>: " + " ".join("%.2f" % x for x in times) + " us")
    ts = np.zeros((nwg, 13), np.uint64)
    _lib.check(rd(ts.ctypes.data, nwg))
    S = ts[:, [0, 10, 11, 1]].astype(np.int64)
    ok = (S > 0).all(1)
    dS = np.diff(S[ok], axis=1)
    for k, name in enumerate(["start -> faces arrived", "faces -> vertices arrived",
                              "vertices -> records computed and stored"]):
        print("  thread 0: %-36s median %7.0f  p90 %7.0f ticks" % (name, np.median(dS[:, k]), np.percentile(dS[:, k], 90)))
    T = ts[:, [0, 1, 2, 3, 7]].astype(np.int64)
    d = np.diff(T, axis=1)
    life = T[:, 4] - T[:, 0]
    tick_us = times[-1] / max(float(np.median(life)), 1.0)
    names = ["records (loads, R1-R5, stores)", "LDS count flush", "slab reservation", "placement (drained)"]
    for k, name in enumerate(names):
        print("  %-32s median %7.0f  p90 %7.0f ticks  (%4.1f%% of the median lifetime)" % (
            name, np.median(d[:, k]), np.percentile(d[:, k], 90), 100.0 * np.median(d[:, k]) / np.median(life)))
    xcc = ts[:, 9].astype(np.int64) & 0xf
    st, en = [], []
    for x in np.unique(xcc):
        m = xcc == x
        t0 = T[m, 0].min()
        st.append(T[m, 0] - t0)
        en.append(T[m, 4] - t0)
    st, en = np.concatenate(st), np.concatenate(en)
    print("  lifetime median %.0f ticks, p90 %.0f; per XCC: starts p50 / p90 / max %.0f / %.0f / %.0f, ends p50 / "
          "max %.0f / %.0f ticks after the XCC's first start" % (
              np.median(life), np.percentile(life, 90), np.median(st), np.percentile(st, 90), st.max(),
              np.median(en), en.max()))


if __name__ == "__main__":
    main()
