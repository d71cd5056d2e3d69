"""Backward with more distinct records per tile than the slot table (64) and more row runs than the LDS
tail buffer holds (the global-memory fallbacks), GPU vs oracle via tests/test_gpu_parity.check_scene."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
from test_gpu_parity import check_scene  # noqa: E402

for C in (1, 3, 7):
    for r in (0.6, 1.0, 1.5):
        check_scene(*scenes.random_triangles(F=30000, W=64, H=48, C=C, radius_px=r, seed=int(r * 10) + C))
        print("ok C=%d r=%.1f" % (C, r))
