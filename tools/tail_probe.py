"""The launch's critical path (round 3): per-block stamps put the longest C3 waves in the top tile rows,
dispatched first and running ~200 us, the whole launch.  This probe times the top tile rows cast alone
(tile_row_start / tile_row_step select them) against the full frame, to split their latency into the
chain itself and contention with the rest of the launch.  usage: python tools/tail_probe.py [--reps 20]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--config", default="c3")
    a = ap.parse_args()
    import torch

    import raytracing_test_amd as rt

    levels, cols, W, H = {"c3": (6, 4096, 1920, 1080), "c5": (7, 16384, 3840, 2160)}[a.config]
    tree = rt.Tree.terrain_gpu(levels, cols, cols, 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    org = (4.0, 90.0, 4.0)
    rows = H // 8
    s = torch.cuda.current_stream()

    def timed(desc, out):
        for _ in range(3):
            tree.cast(desc, out, s)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            tree.cast(desc, out, s)
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return round(statistics.median(ms) * 1e3, 1)

    res = {"config": a.config}
    full = rt.Tree.frame_desc(org, cam, W, H, 16384)
    res["full_us"] = timed(full, rt.Tree.alloc_hits(rt.Tree.count(full), 0))
    for k in (1, 2, 4, 8, 16, 34, 68):
        d = rt.Tree.frame_desc(org, cam, W, H, 16384, tile_row_start=rows - k, tile_row_step=1)
        res["top%d_us" % k] = timed(d, rt.Tree.alloc_hits(rt.Tree.count(d), 0))
    # the bottom half alone (short waves only)
    d = rt.Tree.frame_desc(org, cam, W, H, 16384, tile_row_start=0, tile_row_step=2)
    res["every2nd_row_us"] = timed(d, rt.Tree.alloc_hits(rt.Tree.count(d), 0))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
