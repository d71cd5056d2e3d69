"""Evaluation of per-4x4-sub-block entry lists in the raster, by counting.

For the config-3 scene, counts for every wave block (8x8 pixels, the product's unit) and every 4x4 sub-block
the entries the raster would walk: records whose pixel bbox overlaps the block and none of whose three edges
excludes all of the block's pixel centres (the test stage_tile makes per block, here in float64 on the
window-space vertices -- the same decision up to the snapping, which does not change the averages).  With
one list per 4x4 sub-block, each 16-lane row of a wave walks its own list, so a wave runs max-of-four
iterations instead of the whole block's list.  Prints the averages weighted by work (per wave).

    python tools/sub_block_lists.py            (CPU, ~1 min)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402


def main():
    W = H = 1024
    bg, v, c, f = scenes.random_triangles(F=50000, W=W, H=H, seed=0)
    p = v[f]  # [F, 3, 4]
    xw = (p[..., 0] / p[..., 3] + 1.0) * W / 2
    yw = (p[..., 1] / p[..., 3] + 1.0) * H / 2
    nb8 = np.zeros((H // 8, W // 8), np.int64)
    nb4 = np.zeros((H // 4, W // 4), np.int64)
    for t in range(len(f)):
        X, Y = xw[t], yw[t]
        area = (X[1] - X[0]) * (Y[2] - Y[0]) - (X[2] - X[0]) * (Y[1] - Y[0])
        if area == 0:
            continue
        s = 1.0 if area > 0 else -1.0
        i0, i1 = int(max(np.floor(X.min() - 0.5), 0)), int(min(np.ceil(X.max() - 0.5), W - 1))
        j0, j1 = int(max(np.floor(Y.min() - 0.5), 0)), int(min(np.ceil(Y.max() - 0.5), H - 1))
        if i0 > i1 or j0 > j1:
            continue
        for size, grid in ((8, nb8), (4, nb4)):
            for by in range(j0 // size, j1 // size + 1):
                for bx in range(i0 // size, i1 // size + 1):
                    cx = np.array([bx * size + 0.5, bx * size + size - 0.5])
                    cy = np.array([by * size + 0.5, by * size + size - 0.5])
                    ok = True
                    for k in range(3):
                        a, b = (k + 1) % 3, (k + 2) % 3
                        A, B = s * (Y[a] - Y[b]), s * (X[b] - X[a])
                        C = s * (X[a] * Y[b] - X[b] * Y[a])
                        # the edge's maximum over the block's pixel-centre rectangle
                        if A * (cx[1] if A > 0 else cx[0]) + B * (cy[1] if B > 0 else cy[0]) + C < 0:
                            ok = False
                            break
                    if ok:
                        grid[by, bx] += 1
    # a wave = one 8x8 block; its four 16-lane rows would each own one 4x4 sub-block
    sub = nb4.reshape(H // 8, 2, W // 8, 2).transpose(0, 2, 1, 3).reshape(H // 8, W // 8, 4)
    print("entries per 8x8 block (wave list, product):      mean %.2f" % nb8.mean())
    print("entries per 4x4 sub-block:                       mean %.2f" % nb4.mean())
    print("max over a wave's four 4x4 lists (iterations):   mean %.2f" % sub.max(-1).mean())
    print("sum over a wave's four 4x4 lists (list writes):  mean %.2f" % sub.sum(-1).mean())
    print("iterations saved per wave: %.2f of %.2f (%.0f %%)" % (nb8.mean() - sub.max(-1).mean(), nb8.mean(),
                                                               100 * (1 - sub.max(-1).mean() / nb8.mean())))


if __name__ == "__main__":
    main()
