"""One graph of the public op (py impl) with autograd inside: the scratch's parity / count words before and after
each replay, and the address ranges of the graph's tensors."""
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import scenes  # noqa: E402
from dirt_amd import rasterise_ops  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "grad"
bg, v, c, f = (a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=90))
B, H, W, C = bg.shape
t = [torch.from_numpy(a).cuda().requires_grad_(True) for a in (bg, v, c)]
ft = torch.from_numpy(f).cuda()
g = torch.randn(bg.shape, device="cuda")
s_ = torch.cuda.Stream()
s_.wait_stream(torch.cuda.current_stream())
out = {}


def step():
    px, gb = rasterise_ops._RasteriseFunction.apply(t[0], t[1], t[2], ft, None, H, W, C, 0, 0, False, False)
    out["px"], out["gb"] = px, gb
    if mode == "grad":
        out["grads"] = torch.autograd.grad(px, t, g)


with torch.cuda.stream(s_):
    step()
    ref = out["px"].detach().clone()
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    step()
ws = rasterise_ops._workspace
E0 = list(ws._cap.values())[0]
print("scratch", hex(E0.data_ptr()), E0.numel())
for name, x in [("px", out["px"]), ("gb", out["gb"])] + [("grad%d" % k, x) for k, x in enumerate(out.get("grads", ()))]:
    print(name, hex(x.data_ptr()), x.numel() * x.element_size(),
          "OVERLAPS scratch" if x.data_ptr() < E0.data_ptr() + E0.numel() and E0.data_ptr() < x.data_ptr() + x.numel() * x.element_size() else "")
w = E0.view(torch.int32)
flag = 3072 // 4
for r in range(3):
    print("before replay %d: P %d Q %d counts[0..5] %s" % (r, int(w[flag + 16]), int(w[flag + 32]), [int(w[64 * k]) for k in range(12)]))
    graph.replay()
    torch.cuda.synchronize()
    d = (out["px"] - ref).abs()
    print("replay %d: %d pixels differ" % (r, int((d.amax(-1) > 0).sum())), flush=True)
