"""Re-run one adversarial fuzz seed of tests/test_gpu_parity.py::test_fuzz_adversarial_scenes on the GPU and
print the gradient elements outside the tolerance with what the scene holds there (faces touching the vertex,
their w, clipping, areas).  usage: python tools/debug/fuzz_seed.py SEED"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from oracle import oracle  # noqa: E402

seed = int(sys.argv[1])
W, H = [(64, 48), (33, 17), (130, 70)][seed % 3]
C = 3 if seed < 36 else (3, 7, 1, 5)[seed % 4]
if seed % 4 == 3:
    frames = [scenes.adversarial_scene(seed * 10 + k, W=W, H=H, C=C, F=150) for k in range(2)]
    F = max(fr[3].shape[0] for fr in frames)
    frames = [(bg, v, c, np.concatenate([f, np.zeros((F - f.shape[0], 3), np.int32)])) for bg, v, c, f in frames]
    V = max(fr[1].shape[0] for fr in frames)
    frames = [(bg, np.concatenate([v, np.tile(v[:1], (V - v.shape[0], 1))]),
               np.concatenate([c, np.tile(c[:1], (V - c.shape[0], 1))]), f) for bg, v, c, f in frames]
    bg, v, c, f = [np.stack([fr[k] for fr in frames]) for k in range(4)]
else:
    bg, v, c, f = (a[None] for a in scenes.adversarial_scene(seed, W=W, H=H, C=C))
rng = np.random.default_rng(seed)
gp = rng.standard_normal(bg.shape).astype(np.float32)
g = T.run_gpu(bg, v, c, f, gp)
px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
print("forward bit-exact:", np.array_equal(g["gbuffer"], gb), np.array_equal(g["pixels"], px))
gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, gp, gb)
for name, a, r in (("grad_vertices", g["grad_vertices"], gv), ("grad_colors", g["grad_colors"], gc)):
    scale = np.abs(r).max()
    err = np.abs(a.astype(np.float64) - r)
    tol = T.RTOL * np.abs(r) + T.ATOL_REL * scale
    bad = np.argwhere(~(err <= tol))
    print("%s scale %g, %d outside" % (name, scale, len(bad)))
    for idx in bad[:10]:
        b, vi = int(idx[0]), int(idx[1])
        print("  frame %d vertex %d comp %s: gpu %.6g oracle %.6g err %.3g tol %.3g" %
              (b, vi, tuple(idx[2:]), a[tuple(idx)], r[tuple(idx)], err[tuple(idx)], tol[tuple(idx)]))
        for fi in np.argwhere((f[b] == vi).any(-1))[:, 0]:
            tri = v[b][f[b][fi]]
            vis = int(((gb[b] & ((1 << 30) - 1)) == fi).sum())
            clipped = bool(((gb[b] >= 0) & ((gb[b] & (1 << 30)) != 0) & ((gb[b] & ((1 << 30) - 1)) % max(1, 1) >= 0)).any())
            print("     face %d verts %s w %s visible px %d" % (fi, f[b][fi].tolist(), tri[:, 3].tolist(), vis))
            print("        xyz/w", np.round(tri[:, :3] / tri[:, 3:4], 5).tolist())
