"""Traversal counters of the shaded C3 frame (the SVO_CAST_STATS instance of the shading pass): per pixel
averages, and the per-pixel work of the rays the shading bends (reflected / refracted: their end differs
from the primary ray's) against the others — iterations, lookups, brick steps, ceiling moves.
usage: python tools/shade_stats.py [--cols 4096] [--flags F]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--flags", type=int, default=0)
    a = ap.parse_args()
    import raytracing_test_amd as rt

    solid = rt.Tree.terrain_gpu(6, a.cols, a.cols, 0)
    scene = rt.Tree.terrain_gpu(6, a.cols, a.cols, 0, view=rt.VIEW_ALL)
    dn = rt.normalize([1.0, -0.45, 1.0])
    W, H, S = 1920, 1080, 16384
    st = solid.shade_stats((4.0, 90.0, 4.0), dn, W, H, S, scene=scene, flags=a.flags, ray_work=True)
    rw = st.pop("ray_work").astype(np.uint64)
    look, iters, brick, loads = (rw & 0xFFFF), (rw >> 16) & 0xFFFF, (rw >> 32) & 0xFFFF, (rw >> 48) & 0xFFFF
    _, hits = solid.shade_frame((4.0, 90.0, 4.0), dn, W, H, S, with_hits=True, scene=scene)
    prim = rt.decode_hits(solid.cast_frame((4.0, 90.0, 4.0), dn, W, H, S))
    g = rt.decode_hits(hits)
    bent = ~np.all(g["pos"] == prim["pos"], axis=1)
    res = {"per_pixel": {k: round(v, 3) for k, v in st.items()}, "bent_share": round(float(bent.mean()), 4)}
    for name, sel in (("bent", bent), ("straight", ~bent)):
        res[name] = {"iters": round(float(iters[sel].mean()), 2), "lookups": round(float(look[sel].mean()), 2),
                     "brick_steps": round(float(brick[sel].mean()), 2), "loads": round(float(loads[sel].mean()), 2),
                     "iters_p50_90_99": np.percentile(iters[sel], [50, 90, 99]).round(1).tolist(),
                     "share_of_iters": round(float(iters[sel].sum() / iters.sum()), 4)}
    # the long tail: bent rays at or above their 99th iteration percentile — where they end, how far they went
    sel = bent & (iters >= np.percentile(iters[bent], 99))
    used = np.where(g["hit"], S - g["steps"], S)
    res["bent_tail"] = {"n": int(sel.sum()), "hit_frac": round(float(g["hit"][sel].mean()), 3),
                        "steps_used_p50_90": np.percentile(used[sel], [50, 90]).round(0).tolist(),
                        "end_y_p10_50_90": np.percentile(g["pos"][sel][:, 1], [10, 50, 90]).round(0).tolist(),
                        "lookups": round(float(look[sel].mean()), 1), "brick_steps": round(float(brick[sel].mean()), 1),
                        "prim_y_p50": float(np.median(prim["pos"][sel][:, 1])), "pixel_rows_p10_50_90":
                        np.percentile(np.nonzero(sel)[0] // W, [10, 50, 90]).round(0).tolist()}
    fp = iters.reshape(H // 4, 4, W // 16, 16).transpose(0, 2, 1, 3).reshape(-1, 64).astype(np.float64)
    res["wave_iters_mean_of_max"] = round(float(fp.max(1).mean()), 2)
    res["lane_eff_iters"] = round(float(fp.mean() / fp.max(1).mean()), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
