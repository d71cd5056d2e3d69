"""Forward throughput of the `oceanic_horizon` fragment program on the fork's harness:
full-screen quad, 960x640x3, camera of tests/optimize_horizon.py:285-287.  Compute-bound (VALU: ~110
fixed-polynomial sines per water pixel), so the report is Mpixels/s plus per-kernel microseconds and
the oracle (OpenMP CPU) beside it.  One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402


def main(steps=200, H=640, W=960, B=1, pitch=0.0, shader=1):
    cam_np = np.zeros(16, np.float32)
    cam_np[:8] = [0.0, 200.0, 0.0, pitch, 0.0, 0.0, 0.0, 0.9]
    C = 3
    if shader == 6:  # optical flow: dt, velocity, angular velocity (oceanic_opt_flow.cpp:399-414)
        cam_np[9:16] = [0.5, 10.0, 0.0, 20.0, 0.01, 0.1, -0.02]
    bg = np.zeros((B, H, W, 3), np.float32)
    if shader == 7:  # hill: the harness of tests/square_test.py:14-37 (960x540, 4-channel terrain lookup)
        import scenes
        H, W, C = 540, 960, 4
        cam_np[9:12] = [0.0, 0.0, 3.0]
        bg = np.tile(scenes.hill_terrain(H, W, 4)[None], (B, 1, 1, 1))
    v = np.tile(np.array([[[-1, -1, 0, 1], [-1, 1, 0, 1], [1, 1, 0, 1], [1, -1, 0, 1]]], np.float32), (B, 1, 1))
    f = np.tile(np.array([[[0, 1, 2], [0, 2, 3]]], np.int32), (B, 1, 1))
    c = np.ones((B, 4, C), np.float32)
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(a).to(dev) for a in (bg, v, c, f)]
    cam = torch.from_numpy(cam_np).to(dev)
    sess = RasteriseSession(B, H, W, C, 4, 2, device=dev, shader_id=shader)
    for _ in range(5):
        sess.forward(*t, camera_pos=cam)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            sess.forward(*t, camera_pos=cam)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // 10):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (steps // 10 * 10)
    _lib.profile_enable(True)
    for _ in range(20):
        sess.forward(*t, camera_pos=cam)
    torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.profile_enable(False)
    from oracle import oracle
    nth = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    c0 = time.perf_counter()
    oracle.rasterise_fwd(bg, v, c, f, nthreads=nth, shader_id=shader, camera_pos=cam_np)
    cpu = time.perf_counter() - c0
    names = {1: "oceanic_horizon", 2: "oceanic", 3: "oceanic_still_cloud", 4: "oceanic_no_cloud",
             5: "oceanic_simple_proxy", 6: "oceanic_opt_flow", 7: "hill"}
    print(json.dumps({"metric": "Mpixels/s forward, %s %dx%d full-screen" % (names[shader], W, H), "pitch": pitch, "value":
                      round(B * H * W / dt / 1e6, 1), "ms_per_frame": round(dt * 1e3 / B, 4),
                      "kernels_us": {k: round(ms / n * 1e3, 2) for k, (n, ms) in prof.items() if n},
                      "cpu_oracle": {"Mpixels/s": round(B * H * W / cpu / 1e6, 2), "threads": nth}}))


if __name__ == "__main__":
    main(pitch=float(sys.argv[1]) if len(sys.argv) > 1 else 0.0, shader=int(sys.argv[2]) if len(sys.argv) > 2 else 1)
