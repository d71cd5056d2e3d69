import sys, os
sys.path[:0] = [os.environ.get("GRAFT_REPO_ROOT", "."), os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests")]
import numpy as np, torch, scenes
from oracle import oracle
from dirt_amd import rasterise_ops
bad = 0
for (H, W) in [(17, 1), (17, 2), (17, 3), (20, 1), (33, 1), (17, 16), (17, 17), (32, 1), (16, 1), (1, 17), (18, 5)]:
    for seed in range(6):
        for C in (1, 3):
            bg, v, c, f = scenes.random_triangles(F=60, W=W, H=H, C=C, radius_px=max(2.0, min(W, H) / 2.0), seed=seed * 7 + H + W)
            t = [torch.from_numpy(a[None]).cuda() for a in (bg, v, c, f)]
            p, g = rasterise_ops._rasterise_batched(*t, None, H, W, C, 0, return_gbuffer=True)
            px, gb, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
            gg = g.cpu().numpy()
            if not np.array_equal(gg, gb):
                bad += 1
                idx = np.argwhere(gg != gb)
                print("H=%d W=%d seed=%d C=%d: %d mismatches, first %s gpu %d oracle %d" % (H, W, seed, C, len(idx), idx[0].tolist(), gg[tuple(idx[0])], gb[tuple(idx[0])]))
print("bad", bad)
