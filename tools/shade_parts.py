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


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def work():
    """per-pixel DDA steps of the shaded C3 frame (hit records of the shading pass: a hit used S - stepsLeft
    steps, a miss all S or escaped early), and the per-footprint (16 x 4 wavefront) max against mean"""
    import numpy as np

    solid = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    scene = rt.Tree.terrain_gpu(6, 4096, 4096, 0, view=rt.VIEW_ALL)
    dn = rt.normalize([1.0, -0.45, 1.0])
    W, H, S = 1920, 1080, 16384
    rgba, hits = solid.shade_frame((4.0, 90.0, 4.0), dn, W, H, S, with_hits=True, scene=scene)
    prim = rt.decode_hits(solid.cast_frame((4.0, 90.0, 4.0), dn, W, H, S))
    g = rt.decode_hits(hits)
    used = np.where(g["hit"], S - g["steps"], S).reshape(H, W).astype(np.float64)
    pused = np.where(prim["hit"], S - prim["steps"], S).reshape(H, W).astype(np.float64)
    diff = ~np.all(g["pos"] == prim["pos"], axis=1)
    print("pixels whose shaded ray differs from the primary (reflected / refracted): %.4f" % diff.mean())
    print("steps used per pixel: primary mean %.0f, shaded mean %.0f; shaded percentiles 50/90/99/99.9: %s"
          % (pused.mean(), used.mean(), np.percentile(used, [50, 90, 99, 99.9]).round()))
    fp = used.reshape(H // 4, 4, W // 16, 16).transpose(0, 2, 1, 3).reshape(-1, 64)
    print("per-footprint: mean of means %.0f, mean of maxima %.0f (lane efficiency %.3f); footprints whose max > 4x mean: %.3f"
          % (fp.mean(), fp.max(1).mean(), fp.mean() / fp.max(1).mean(), (fp.max(1) > 4 * fp.mean(1)).mean()))
    big = used.reshape(-1)[diff] if diff.any() else np.zeros(1)
    print("refracted / reflected pixels: steps used mean %.0f, share of all shaded steps %.3f" % (big.mean(), big.sum() / used.sum()))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "work":
    work()
