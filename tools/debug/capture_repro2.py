"""The body of tests/test_gpu_batch_multigpu.py::test_two_graphs_same_layout_second_replayed_first with progress
prints and optional parts switched off (argv: impl, then flags: nojunk, noclear, norefs)."""
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import scenes  # noqa: E402
from dirt_amd import rasterise_ops  # noqa: E402

impl, flags = sys.argv[1], set(sys.argv[2:])
ext = rasterise_ops._torch_ext()


def _gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def op(t0, t1, t2, ft, H, W, C):
    args = (t0, t1, t2, ft, None, H, W, C, 0, 0, False, False)
    return ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args)


if "noclear" not in flags:
    rasterise_ops.workspace_cache_clear(force=True)
if "nojunk" not in flags:
    junk = [torch.full((1 << 22,), 0x01010101, dtype=torch.int32, device="cuda") for _ in range(16)]
    del junk
scenes_ = [tuple(a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=s))
           for s in (90, 91)]
B, H, W, C = scenes_[0][0].shape
graphs, outs = [], []
for k, (bg, v, c, f) in enumerate(scenes_):
    t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
    ft = _gpu(f)
    g = torch.randn(bg.shape, device="cuda")
    if "norefs" not in flags:
        if "refs_side" in flags:
            sr = torch.cuda.Stream()
            sr.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(sr):
                px, _ = op(t[0], t[1], t[2], ft, H, W, C)
                ref = torch.autograd.grad(px, t, g)
            torch.cuda.synchronize()
        elif "refs_nograd" in flags:
            px, _ = op(t[0].detach(), t[1].detach(), t[2].detach(), ft, H, W, C)
        else:
            px, _ = op(t[0], t[1], t[2], ft, H, W, C)
            ref = torch.autograd.grad(px, t, g)
        print(k, "refs ok", flush=True)
    out = {}

    if "plain_capture" in flags:
        def step(t=t, ft=ft, g=g, out=out):
            out["y"] = (t[0] * 2).sum()
    else:
      def step(t=t, ft=ft, g=g, out=out):
        px, _ = op(t[0], t[1], t[2], ft, H, W, C)
        out["px"] = px
        out["grads"] = torch.autograd.grad(px, t, g)

    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        step()
    torch.cuda.current_stream().wait_stream(s_)
    torch.cuda.synchronize()
    print(k, "warm ok", flush=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    print(k, "capture ok", flush=True)
    graphs.append(graph)
    outs.append(out)
torch.cuda.synchronize()
for k in (1, 0):
    graphs[k].replay()
    torch.cuda.synchronize()
print("replays ok", flush=True)
