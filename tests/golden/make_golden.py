"""Regenerate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference ships no golden vectors and cannot run here (TF1 + NVIDIA EGL/GL + CUDA), so
these fixtures pin the oracle's restatement of the reference semantics over time; the analytic
known-answer tests in tests/test_oracle.py pin the oracle itself against the reference's README and
tests.  Each fixture holds the op inputs, the forward outputs (pixels, g-buffer) and the backward
outputs for a seeded grad_pixels.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]

import scenes  # noqa: E402
from oracle import oracle  # noqa: E402


def cases():
    yield "readme_square", scenes.readme_square()
    yield "cube_256", scenes.cube_scene()
    yield "cylinder_48x36", scenes.cylinder_scene()
    yield "random512_64x64", scenes.random_triangles(F=512, W=64, H=64, radius_px=10.0, seed=0)
    yield "perspective_96x80", scenes.random_triangles(F=300, W=96, H=80, radius_px=10.0, seed=5, perspective=True)
    yield "clipping_96x64", scenes.clipping_scene()
    yield "shared_mesh_80x60", scenes.shared_mesh_scene()


def make(name, scene):
    bg, v, c, f = (a[None] for a in scene)
    px, gb, st = oracle.rasterise_fwd(bg, v, c, f, nthreads=1)
    assert st == 0
    # a few exactly representable levels: compresses well, still exercises every sign/magnitude path
    gp = (np.random.default_rng(12345).integers(-4, 5, size=px.shape) * 0.25).astype(np.float32)
    gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, gp, gb, nthreads=1)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), background=bg, vertices=v, vertex_colors=c, faces=f,
                        pixels=px, gbuffer=gb, grad_pixels=gp, grad_vertices=gv, grad_vertex_colors=gc,
                        grad_background=gbg)


if __name__ == "__main__":
    for name, scene in cases():
        make(name, scene)
        print("wrote", name)
