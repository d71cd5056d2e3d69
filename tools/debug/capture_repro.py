"""Repro of the capture_end segfault (round 5): variants of capturing the public op + autograd into graphs.
usage: python tools/debug/capture_repro.py VARIANT IMPL   (run each in its own process)"""
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import scenes  # noqa: E402
from dirt_amd import rasterise_ops  # noqa: E402

variant, impl = sys.argv[1], sys.argv[2]
ext = rasterise_ops._torch_ext()


def op(t0, t1, t2, ft, H, W, C):
    args = (t0, t1, t2, ft, None, H, W, C, 0, 0, False, False)
    return ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args)


bg, v, c, f = (a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=90))
B, H, W, C = bg.shape
t = [torch.from_numpy(a).cuda().requires_grad_(True) for a in (bg, v, c)]
ft = torch.from_numpy(f).cuda()
g = torch.randn(bg.shape, device="cuda")
out = {}


def step(grad=True):
    px, _ = op(t[0], t[1], t[2], ft, H, W, C)
    out["px"] = px
    if grad:
        out["grads"] = torch.autograd.grad(px, t, g)


s_ = torch.cuda.Stream()
s_.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s_):
    step()
torch.cuda.current_stream().wait_stream(s_)
torch.cuda.synchronize()
print("warm ok", flush=True)
graph = torch.cuda.CUDAGraph()
if variant == "fwd_only_default_stream":
    with torch.cuda.graph(graph):
        step(grad=False)
elif variant == "fwdbwd_default_stream":
    with torch.cuda.graph(graph):
        step()
elif variant == "fwdbwd_side_stream":
    with torch.cuda.graph(graph, stream=s_):
        step()
elif variant == "fwdbwd_side_stream_nowarm_samestream":
    s2 = torch.cuda.Stream()
    with torch.cuda.graph(graph, stream=s2):
        step()
elif variant in ("two_default", "two_default_clear_between"):
    with torch.cuda.graph(graph):
        step()
    print("capture 1 ok", flush=True)
    if variant == "two_default_clear_between":
        rasterise_ops.workspace_cache_clear(force=True)
    with torch.cuda.stream(s_):
        step()
    torch.cuda.current_stream().wait_stream(s_)
    torch.cuda.synchronize()
    graph2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph2):
        step()
    print("capture 2 ok", flush=True)
    graph2.replay()
print("capture ok", flush=True)
graph.replay()
torch.cuda.synchronize()
print("replay ok", flush=True)
