"""Control experiment for the capture_end segfault.

The sequence of tests/test_gpu_batch_multigpu.py::test_two_graphs_same_layout_second_replayed_first, one graph:
an eager forward + torch.autograd.grad on the legacy default stream, a warm-up of the same step on a side stream,
then torch.cuda.graph capture of the step on torch.cuda.graph's own capture stream.

    python tools/debug/capture_control.py IMPL MODE
    IMPL: ext   -- the op's C++ autograd function (dirt_amd/_dirt_torch)
          py    -- the op's Python torch.autograd.Function
          torch -- no dirt_amd code at all: px = bg * 0.5 + 1e-3 * (v.sum() + c.sum()), the same leaves and shapes
    MODE: kept     -- the eager reference's output (and so its autograd graph and the leaves' AccumulateGrad nodes,
                      created on the default stream) stays alive through the capture, as in the round-5 test
          released -- `del px` after the reference and the warm-up's outputs dropped before the capture (what
                      torch's AccumulateGrad stream-mismatch warning asks for)

Prints one line per stage; a crash shows as the last stage reached.
"""
import faulthandler
import os
import sys
import warnings

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import scenes  # noqa: E402

impl, mode = sys.argv[1], sys.argv[2]
assert impl in ("ext", "py", "torch") and mode in ("kept", "released")

if impl != "torch":
    from dirt_amd import rasterise_ops
    ext = rasterise_ops._torch_ext()


def op(t0, t1, t2, ft, H, W, C):
    if impl == "torch":
        return t0 * 0.5 + 1e-3 * (t1.sum() + t2.sum())
    args = (t0, t1, t2, ft, None, H, W, C, 0, 0, False, False)
    return (ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args))[0]


def main():
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=2500, W=160, H=128, radius_px=10.0, seed=90))
    B, H, W, C = bg.shape
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda().requires_grad_(True) for a in (bg, v, c)]
    ft = torch.from_numpy(np.ascontiguousarray(f)).cuda()
    g = torch.randn(bg.shape, device="cuda")
    with warnings.catch_warnings(record=True) as wlist:
        warnings.simplefilter("always")
        px = op(t[0], t[1], t[2], ft, H, W, C)  # eager reference on the legacy default stream
        ref = [x.clone() for x in torch.autograd.grad(px, t, g)]
        if mode == "released":
            del px
        print("reference ok", flush=True)
        out = {}

        def step():
            y = op(t[0], t[1], t[2], ft, H, W, C)
            out["px"] = y
            out["grads"] = torch.autograd.grad(y, t, g)

        s_ = torch.cuda.Stream()
        s_.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_):
            step()
        torch.cuda.current_stream().wait_stream(s_)
        torch.cuda.synchronize()
        if mode == "released":
            out.clear()
        print("warm-up ok", flush=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        print("capture ok", flush=True)
        graph.replay()
        torch.cuda.synchronize()
        same = all(torch.allclose(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()) + 1e-30)
                   for a, b in zip(out["grads"], ref))
        print("replay ok, gradients equal the eager reference: %s" % same, flush=True)
    mism = [w for w in wlist if "AccumulateGrad node's stream does not match" in str(w.message)]
    print("AccumulateGrad stream-mismatch warnings: %d" % len(mism), flush=True)


main()
