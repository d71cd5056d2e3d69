"""Two graphs of the public op (same layout, torch.cuda.graph's default capture stream): which replays match the
eager result?  argv: impl, order (e.g. 0101 / 1010 / 00), [one] = capture only graph 0"""
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

impl, order = sys.argv[1], sys.argv[2]
flags = set(sys.argv[3:])
KEEP = []
if "keep_saved" in flags:
    _orig_sfb = torch.autograd.function.FunctionCtx.save_for_backward

    def _sfb(self, *ts):
        KEEP.extend(ts)
        return _orig_sfb(self, *ts)
    torch.autograd.function.FunctionCtx.save_for_backward = _sfb
ext = rasterise_ops._torch_ext()


def op(t0, t1, t2, ft, H, W, C):
    args = (t0, t1, t2, ft, None, H, W, C, 0, 0, False, False)
    return ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args)


scenes_ = [tuple(a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=s))
           for s in (90, 91)]
B, H, W, C = scenes_[0][0].shape
graphs, outs, refs = [], [], []
graph_inputs = []
for k, (bg, v, c, f) in enumerate(scenes_):
    t = [torch.from_numpy(a).cuda().requires_grad_(True) for a in (bg, v, c)]
    ft = torch.from_numpy(f).cuda()
    g = torch.randn(bg.shape, device="cuda")
    if k == 0:
        graph_inputs = t + [ft, g]
    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        px, _ = op(t[0], t[1], t[2], ft, H, W, C)
        refs.append(px.detach().clone())
        gr = torch.autograd.grad(px, t, g)
    torch.cuda.synchronize()
    out = {}

    def step(t=t, ft=ft, g=g, out=out):
        px, gb = op(t[0], t[1], t[2], ft, H, W, C)
        out["px"] = px
        out["gb"] = gb
        if "nograd" not in flags:
            out["grads"] = torch.autograd.grad(px, t, g)

    with torch.cuda.stream(s_):
        step()
    torch.cuda.current_stream().wait_stream(s_)
    torch.cuda.synchronize()
    if k == 1 and "one" in flags:
        break
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    graphs.append(graph)
    outs.append(out)
torch.cuda.synchronize()
inputs0 = [x.detach().clone() for x in graph_inputs] if "check_inputs" in flags else None
for ch in order:
    k = int(ch)
    graphs[k].replay()
    torch.cuda.synchronize()
    d = (outs[k]["px"] - refs[k]).abs()
    print("replay graph %d: max|diff| %.3g, %d pixels differ" % (k, float(d.max()), int((d.amax(-1) > 0).sum())), flush=True)
    if inputs0 is not None:
        print("   inputs of graph 0 intact:", [bool(torch.equal(a, b.detach())) for a, b in zip(inputs0, graph_inputs)])
    if impl == "py" and "scratch" in flags:
        E = list(rasterise_ops._workspace._cap.values())
        w = E[0].view(torch.int32) if E else None
        if w is not None:
            print("   scratch P %d Q %d counts %s" % (int(w[768 + 16]), int(w[768 + 32]), [int(w[64 * q]) for q in range(12)]))
