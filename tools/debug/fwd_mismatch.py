"""Dump one fuzz seed's scene with the GPU and oracle forward outputs where their g-buffers differ
(gpurun_out/fwd_mismatch_SEED.npz) for host-side analysis.  usage: python tools/debug/fwd_mismatch.py SEED"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from oracle import oracle  # noqa: E402

seed = int(sys.argv[1])
bg, v, c, f = scenes.fuzz_case(seed)
g = T.run_gpu(bg, v, c, f, None)
px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
bad = np.argwhere(g["gbuffer"] != gb)
print("seed %d: shape %s, %d g-buffer words differ" % (seed, bg.shape, len(bad)))
for b, y, x in bad:
    print("  frame %d row %d col %d: gpu %d oracle %d" % (b, y, x, g["gbuffer"][b, y, x], gb[b, y, x]))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "fwd_mismatch_%d.npz" % seed), bg=bg, v=v, c=c, f=f,
         gpu_gb=g["gbuffer"], gpu_px=g["pixels"], ref_gb=gb, ref_px=px)
