"""Critical-path probe (round 5): does a far-field wave finish sooner when it carries fewer rays?  The top K tile rows of
the C3 frame are cast as explicit rays (the same pixel directions, footprint by footprint as frame mode lays them out),
L real rays per 64-lane wave and 64 - L steep filler rays (normalize(0.01, -1, 0.01): a few iterations each) — so a
wave's lanes diverge over fewer paths per iteration.  Times each (K, L) launch (HIP events, median of --reps) and the
full frame in frame mode for reference.  usage: python tools/lane_probe.py [--reps 15]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--ks", default="4,16,34,135")
    ap.add_argument("--ls", default="64,32,16")
    a = ap.parse_args()
    import numpy as np
    import torch

    import raytracing_test_amd as rt

    W, H, S = 1920, 1080, 16384
    tree = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    org = (4.0, 90.0, 4.0)
    dirs = rt.pixel_dirs(cam, W, H)  # (H, W, 3), rows from the bottom
    filler = rt.normalize((0.01, -1.0, 0.01))
    s = torch.cuda.current_stream()

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(400000)  # (keeps the GPU busy while the host prepares the launch: host time stays out of e0..e1)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return round(statistics.median(ms) * 1e3, 1)

    rows = H // 8
    res = {}
    full = rt.Tree.frame_desc(org, cam, W, H, S)
    fo = rt.Tree.alloc_hits(rt.Tree.count(full), 0)
    res["frame_full_us"] = timed(lambda: tree.cast(full, fo, s))
    lane = np.arange(64)
    for k in [int(x) for x in a.ks.split(",")]:
        # footprints of the top k tile rows in frame-mode dispatch order: tile row from the top, then 16x4 footprints
        fps = []
        for t in range(k):
            tr = rows - 1 - t
            for tx in range(2 * (W // 16)):
                rr = ((tx & 1) << 2) + (lane >> 4)
                px = ((tx >> 1) << 4) + (lane & 15)
                py = tr * 8 + rr
                fps.append(dirs[py, px])
        fps = np.stack(fps)  # (n_fp, 64, 3)
        d = rt.Tree.frame_desc(org, cam, W, H, S, tile_row_start=rows - k, tile_row_step=1)
        do = rt.Tree.alloc_hits(rt.Tree.count(d), 0)
        res["frame_top%d_us" % k] = timed(lambda: tree.cast(d, do, s))
        for L in [int(x) for x in a.ls.split(",")]:
            waves = fps.reshape(-1, L, 3)  # L consecutive rays of a footprint per wave
            buf = np.empty((waves.shape[0], 64, 3), np.float32)
            buf[:, :L] = waves
            buf[:, L:] = filler
            dv = torch.from_numpy(buf.reshape(-1, 3)).cuda()
            out = rt.Tree.alloc_hits(dv.shape[0], 0)
            res["explicit_top%d_L%d_us" % (k, L)] = timed(lambda: tree.cast_rays(dv, steps=S, origin=org, out=out, stream=s, sync=False))
        print(json.dumps(res), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
