"""Is the backward's drain tail set by per-tile work or by when a workgroup starts?  (config 3)

Runs the instrumented backward (variant 128, per-workgroup timestamps, as tools/phase_ts.py) and relates each
workgroup's lifetime to its tile's content, computed on the host from the forward's g-buffer: distinct records
in the 18x18 tile + halo region (the slot table's size) and covered pixels.  Prints the correlations, the
lifetime by start order on its CU (first vs second round of 8), and where the per-CU last finishers sit in
the tile-cost distribution -- a heavy-first tile order can only shorten the tail if those are heavy tiles."""
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


def xcd_tile(x, n):
    q, r, g, k = n >> 3, n & 7, x & 7, x >> 3
    return g * q + np.minimum(g, r) + k


def tile_content(gb, H, W, T=16):
    """per tile (row-major): distinct record words and covered pixels over the tile + one-pixel halo"""
    ntx, nty = (W + T - 1) // T, (H + T - 1) // T
    img = gb[::-1]  # g-buffer rows are stored bottom-up (row H-1-j holds pixel row j)
    pad = np.full((H + 2, W + 2), -1, np.int64)
    pad[1:-1, 1:-1] = img
    nrec = np.zeros(ntx * nty, np.int64)
    ncov = np.zeros(ntx * nty, np.int64)
    for ty in range(nty):
        for tx in range(ntx):
            reg = pad[ty * T:ty * T + T + 2, tx * T:tx * T + T + 2]
            u = np.unique(reg)
            nrec[ty * ntx + tx] = (u >= 0).sum()
            ncov[ty * ntx + tx] = (reg[1:-1, 1:-1] >= 0).sum()
    return nrec, ncov


def main():
    dev = torch.device("cuda", 0)
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
    print("instrumented backward %.2f us" % (ms.value * 1e3))
    ts = np.zeros((nwg, 13), np.uint64)
    _lib.check(rd(ts.ctypes.data, nwg))
    T = ts[:, :8].astype(np.int64)
    hw = ts[:, 8].astype(np.int64)
    xcc = ts[:, 9].astype(np.int64) & 0xf
    key = ((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 0xf)
    for x in np.unique(key):
        m = key == x
        T[m] -= T[m, 0].min()
    life = (T[:, 7] - T[:, 0]).astype(np.float64)
    tiles = xcd_tile(np.arange(nwg), nwg)
    nrec, ncov = tile_content(sess.gbuffer[0].cpu().numpy().astype(np.int64), H, W)
    r_rec, r_cov = nrec[tiles], ncov[tiles]
    print("tile records (18x18 region): mean %.1f  p10 %d  p90 %d  max %d" % (
        r_rec.mean(), np.percentile(r_rec, 10), np.percentile(r_rec, 90), r_rec.max()))
    print("corr(lifetime, records) %.3f   corr(lifetime, covered px) %.3f" % (
        np.corrcoef(life, r_rec)[0, 1], np.corrcoef(life, r_cov)[0, 1]))
    # start order on its CU
    order = np.zeros(nwg, np.int64)
    for x in np.unique(key):
        idx = np.where(key == x)[0]
        order[idx[np.argsort(T[idx, 0], kind="stable")]] = np.arange(len(idx))
    first = order < 8
    print("lifetime median: first 8 on a CU %.0f ticks, later %.0f ticks; corr(lifetime, start) %.3f" % (
        np.median(life[first]), np.median(life[~first]), np.corrcoef(life, T[:, 0])[0, 1]))
    # residual after the content model
    A = np.stack([np.ones(nwg), r_rec, r_cov, first.astype(np.float64)], 1)
    coef, *_ = np.linalg.lstsq(A, life, rcond=None)
    pred = A @ coef
    print("lifetime ~ %.0f + %.1f*records + %.2f*covered + %.0f*first_round: R^2 %.3f" % (
        coef[0], coef[1], coef[2], coef[3], 1 - ((life - pred) ** 2).sum() / ((life - life.mean()) ** 2).sum()))
    # the per-CU last finisher
    lasts = []
    for x in np.unique(key):
        idx = np.where(key == x)[0]
        lasts.append(idx[np.argmax(T[idx, 7])])
    lasts = np.array(lasts)
    pct = np.array([(r_rec < r_rec[k]).mean() for k in lasts])
    print("per-CU last finishers: records percentile median %.2f (0.5 = typical tile), start order median %.0f" % (
        np.median(pct), np.median(order[lasts])))
    ends = np.array([T[key == x, 7].max() for x in np.unique(key)])
    span = np.median(ends)
    gap = np.array([T[key == x, 7].max() - np.sort(T[key == x, 7])[-8] for x in np.unique(key)])
    print("per-CU span median %.0f ticks; last end - 8th-last end median %.0f ticks (%.1f %% of the span)" % (
        span, np.median(gap), 100 * np.median(gap) / span))


if __name__ == "__main__":
    main()
