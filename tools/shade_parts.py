"""Where the shading pass spends its time (C3 scene, full view with water): the plain cast, the shaded
frame with and without its shadow rays.  usage: python tools/shade_parts.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracing_test_amd as rt  # noqa: E402


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    solid = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    scene = rt.Tree.terrain_gpu(6, 4096, 4096, 0, view=rt.VIEW_ALL)
    dn = rt.normalize([1.0, -0.45, 1.0])
    W, H, S = 1920, 1080, 16384
    d = solid.frame_desc((4.0, 90.0, 4.0), dn, W, H, S)
    n = solid.count(d)
    out = solid.alloc_hits(n, 0)
    rgba = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    print("cast            %.4f ms" % timed(lambda: solid.cast(d, out)))
    for sh in (0, 75):
        print("shade shadow=%-3d %.4f ms" % (sh, timed(lambda: solid.shade(d, rgba, shadow_steps=sh, scene=scene))))
    print("shade no water  %.4f ms" % timed(lambda: solid.shade(d, rgba, shadow_steps=75)))


if __name__ == "__main__":
    main()
