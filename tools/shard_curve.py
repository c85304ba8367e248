"""Per-rank cost of strong scaling, measured on one GPU: the fused cast
(svo_cast_wire, 8-B records) of every rank's tile-row shard of one frame for N = 1, 2, 4, 8 ranks
(tile_row_start = r, tile_row_step = N), one launch at a time and with two launches in flight
(consecutive launches alternating between two streams, as a renderer keeps frames in flight).  The
step time of an N-rank strong-scaling run is the slowest rank's, so each N reports the max over its
ranks next to the ideal (the whole frame / N).  HIP events on the launch streams, median of --reps.
usage: python tools/shard_curve.py [--config c5|c3] [--reps 20] [--ns 1,2,4,8] [--flags F]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--inflight-launches", type=int, default=20)
    a = ap.parse_args()
    import torch

    import raytracing_test_amd as rt

    levels, cols, W, H = {"c5": (7, 16384, 3840, 2160), "c3": (6, 4096, 1920, 1080)}[a.config]
    tree = rt.Tree.terrain_gpu(levels, cols, cols, 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    org = (4.0, 90.0, 4.0)
    ppx, ppy = rt.proj_plane(W, H)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()

    def desc(r, n):
        return rt.Tree.frame_desc(org, cam, W, H, 16384, ppx, ppy, tile_row_start=r, tile_row_step=n, flags=a.flags)

    def one_at_a_time(d, buf):
        for _ in range(3):
            tree.cast_wire(d, buf, None, s0)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            tree.cast_wire(d, buf, None, s0)
            e1.record(s0)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return statistics.median(ms) * 1e3  # us

    def in_flight(d, bufs):
        k = a.inflight_launches
        for i in range(4):
            tree.cast_wire(d, bufs[i & 1], None, (s0, s1)[i & 1])
        torch.cuda.synchronize()
        res = []
        for _ in range(max(3, a.reps // 4)):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(s0)
            s1.wait_event(e0)
            for i in range(k):
                tree.cast_wire(d, bufs[i & 1], None, (s0, s1)[i & 1])
            e1.record(s1)
            s0.wait_event(e1)
            e2.record(s0)
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e2) / k)
        return statistics.median(res) * 1e3  # us per launch

    out = {"config": a.config, "frame": [W, H], "flags": a.flags, "how": "svo_cast_wire of rank r's tile rows (r mod N); median of %d "
           "launches one at a time; in flight: %d consecutive launches alternating two streams, per launch" % (a.reps, a.inflight_launches),
           "curve": []}
    full_us = None
    for n in [int(x) for x in a.ns.split(",")]:
        per = []
        per_if = []
        for r in range(n):
            d = desc(r, n)
            cnt = rt.Tree.count(d)
            wb = tree.wire_bytes(d)
            bufs = [torch.empty((cnt, wb), dtype=torch.uint8, device="cuda") for _ in range(2)]
            per.append(one_at_a_time(d, bufs[0]))
            per_if.append(in_flight(d, bufs))
            del bufs
        if n == 1:
            full_us = per[0]
        row = {"n": n, "rank_us": [round(x, 1) for x in per], "max_us": round(max(per), 1), "ideal_us": round(full_us / n, 1),
               "eff": round(full_us / n / max(per), 3), "inflight_rank_us": [round(x, 1) for x in per_if],
               "inflight_max_us": round(max(per_if), 1),
               "rays_per_s_at_max": round(W * H / (max(per) * 1e-6) / 1e9, 2),
               "rays_per_s_inflight": round(W * H / (max(per_if) * 1e-6) / 1e9, 2)}
        out["curve"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
