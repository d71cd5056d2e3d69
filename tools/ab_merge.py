"""A/B of the backward's shared-vertex flush merge (grad_kernel MERGE, DIRT_GRAD_MERGE=0 / 1), interleaved
rounds in one process: bench_configs' graph-replayed fwd+bwd steps and per-kernel event times, the c4 deferred
chain, and the gradient difference between the two settings (float summation order only).

    python tools/ab_merge.py [rounds]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]
os.environ["DIRT_NO_CPU"] = "1"
import bench_configs as bc  # noqa: E402
import scenes  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

SEL = ["c4_deferred20k_512x512x7", "c2_cube_4096x4096x3", "c3_random50k_1024x1024x3",
       "c5_batch8x20k_1024x1024x3_per_gpu"]


def grads(name, merge):
    os.environ["DIRT_GRAD_MERGE"] = str(merge)
    import numpy as np
    frames = bc.CONFIGS[name]()
    host = [np.stack([fr[k] for fr in frames]) for k in range(4)]
    dev = torch.device("cuda", 0)
    bg, v, c, f = (torch.from_numpy(a).to(dev) for a in host)
    B, H, W, C = bg.shape
    torch.manual_seed(0)
    g = torch.randn((B, H, W, C), device=dev)
    sess = RasteriseSession(B, H, W, C, v.shape[1], f.shape[1], device=dev)
    sess.forward(bg, v, c, f)
    out = sess.backward(g)
    torch.cuda.synchronize()
    return [o.clone() for o in out if o is not None]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for name in SEL:
        a, b = grads(name, 0), grads(name, 1)
        rel = [float((x - y).abs().max() / y.abs().max().clamp_min(1e-30)) for x, y in zip(a, b)]
        print(json.dumps({"config": name, "grad_rel_diff_merge_vs_not": rel}), flush=True)
    for r in range(rounds):
        for merge in (0, 1):
            os.environ["DIRT_GRAD_MERGE"] = str(merge)
            for name in SEL:
                res = bc.run(name, bc.CONFIGS[name]())
                print(json.dumps({"round": r, "merge": merge, "config": name,
                                  "Mpix_s": res["Mpixels_per_s_fwd_bwd"], "us_per_step": res["us_per_step"],
                                  "kernels_us": res["kernels_us"]}), flush=True)
            ch = bc.deferred_chain()
            print(json.dumps({"round": r, "merge": merge, "config": "c4_chain",
                              "ms_graph": ch.get("ms_per_step_graph"), "ms_eager": ch["ms_per_step_eager"]}),
                  flush=True)
    os.environ.pop("DIRT_GRAD_MERGE", None)


if __name__ == "__main__":
    main()
