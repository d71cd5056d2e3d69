"""Frame-size sweep (GPU vs oracle, tests/test_gpu_parity.check_scene): every failure is printed.

    python tools/debug/size_sweep.py
"""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
from test_gpu_parity import check_scene  # noqa: E402

rng = np.random.default_rng(123)
sizes = [(h, w) for h in (1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 129) for w in (1, 3, 16, 17, 33, 64, 65, 130)]
sizes += [(int(a), int(b)) for a, b in rng.integers(1, 700, size=(40, 2))]
bad = 0
for k, (H, W) in enumerate(sizes):
    C = (1, 3, 7)[k % 3]
    B = 1 + (k % 4 == 0)
    cap = 0
    try:
        frames = [scenes.random_triangles(F=int(rng.integers(0, 400)) if b == 0 else 0, W=W, H=H, C=C,
                                          radius_px=float(rng.uniform(1.0, 40.0)), seed=k * 10 + b,
                                          perspective=bool(k % 2)) for b in range(B)]
        F = max(fr[3].shape[0] for fr in frames)
        if F == 0:
            continue
        frames = [scenes.random_triangles(F=F, W=W, H=H, C=C, radius_px=float(rng.uniform(1.0, 40.0)),
                                          seed=k * 10 + b, perspective=bool(k % 2)) for b in range(B)]
        cap = int(rng.integers(1, 24)) if k % 3 == 1 else 0  # every third size: tiny slabs (overflow path)
        check_scene(*[np.stack([fr[j] for fr in frames]) for j in range(4)], seed=k, bin_capacity=cap)
    except Exception as e:  # noqa: BLE001
        bad += 1
        print("FAIL H=%d W=%d C=%d B=%d cap=%d: %s" % (H, W, C, B, cap, str(e).splitlines()[0][:200]))
print("sizes", len(sizes), "bad", bad)

# random-index meshes: arbitrary vertex sharing, repeated indices (degenerate faces), V unrelated to F
bad2 = 0
for k in range(60):
    H, W = (int(x) for x in rng.integers(1, 300, size=2))
    C = (1, 3, 7)[k % 3]
    V = int(rng.integers(3, 2000))
    F = int(rng.integers(1, 1500))
    w = rng.uniform(0.5, 2.0, size=(V, 1)) if k % 2 else np.ones((V, 1))
    xy = rng.uniform(-1.3, 1.3, size=(V, 2)) * w
    z = rng.uniform(-1.1, 1.1, size=(V, 1)) * w
    v = np.concatenate([xy, z, w], 1).astype(np.float32)
    f = rng.integers(0, V, size=(F, 3)).astype(np.int32)
    c = rng.uniform(0, 1, size=(V, C)).astype(np.float32)
    bg = rng.uniform(0, 1, size=(H, W, C)).astype(np.float32)
    try:
        check_scene(bg, v, c, f, seed=k)
    except Exception as e:  # noqa: BLE001
        bad2 += 1
        print("FAIL mesh H=%d W=%d C=%d V=%d F=%d: %s" % (H, W, C, V, F, str(e).splitlines()[0][:200]))
print("random-index meshes 60 bad", bad2)
