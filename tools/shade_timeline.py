"""Per-block timeline of the shaded C3 frame (the shading pass with SVO_CAST_TIMELINE: every 64-lane block's start / end
stamp, 100 MHz): the launch's span, how full it stays, the longest blocks and where they sit in the dispatch order, and
which blocks end last — is the frame bound by its longest (lake) waves or by its total work?
usage: python tools/shade_timeline.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import raytracing_test_amd as rt

    solid = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    scene = rt.Tree.terrain_gpu(6, 4096, 4096, 0, view=rt.VIEW_ALL)
    cam = rt.normalize((1.0, -0.45, 1.0))
    W, H, S = 1920, 1080, 16384
    d = solid.frame_desc((4.0, 90.0, 4.0), cam, W, H, S)
    n, nblk = solid.count(d), solid.blocks(d)
    rgba = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    for _ in range(3):
        solid.shade(d, rgba, scene=scene)
    d.flags |= rt.CAST_TIMELINE
    st = torch.zeros(rt.STATS_HEADER + 2 * nblk, dtype=torch.int64, device="cuda")
    d.stats = st.data_ptr()
    solid.shade(d, rgba, scene=scene)
    torch.cuda.synchronize()
    s = st[rt.STATS_HEADER:].cpu().numpy().reshape(-1, 2).astype(np.float64) / 100.0
    t0 = s[:, 0].min()
    beg, end = s[:, 0] - t0, s[:, 1] - t0
    dur = end - beg
    span = end.max()
    bins = np.linspace(0, span, 21)
    live = [int(((beg < b1) & (end > b0)).sum()) for b0, b1 in zip(bins[:-1], bins[1:])]
    order = np.argsort(-dur)
    tiles_x = (W + 15) // 16 * 2  # (16 x 4 footprints: two per 8-pixel tile row per 16 columns)
    res = {"span_us": round(span, 1), "blocks": int(nblk), "mean_block_us": round(float(dur.mean()), 1),
           "packed_us_at_5_waves_per_simd": round(float(dur.sum()) / (256 * 4 * 5), 1),
           "live_blocks_per_20th": live,
           "longest": [{"block": int(b), "start": round(float(beg[b]), 1), "dur": round(float(dur[b]), 1),
                        "dispatch_row": int(b // tiles_x)} for b in order[:12]],
           "last_to_end": [{"block": int(b), "start": round(float(beg[b]), 1), "end": round(float(end[b]), 1),
                            "dispatch_row": int(b // tiles_x)} for b in np.argsort(-end)[:8]],
           "dur_quantiles_50_90_99_999": np.percentile(dur, [50, 90, 99, 99.9]).round(1).tolist(),
           "mean_dur_per_tenth_of_dispatch": [round(float(x.mean()), 1) for x in np.array_split(dur, 10)]}
    print(json.dumps(res), flush=True)
    out = sys.argv[1] if len(sys.argv) > 1 else None
    if out:  # the raw per-block (start, end) of the shaded and the primary frame, for schedule simulations
        d2 = solid.frame_desc((4.0, 90.0, 4.0), cam, W, H, S)
        hits = solid.alloc_hits(n, 0)
        for _ in range(3):
            solid.cast(d2, hits)
        d2.flags |= rt.CAST_TIMELINE
        st2 = torch.zeros(rt.STATS_HEADER + 2 * solid.blocks(d2), dtype=torch.int64, device="cuda")
        d2.stats = st2.data_ptr()
        solid.cast(d2, hits)
        torch.cuda.synchronize()
        p = st2[rt.STATS_HEADER:].cpu().numpy().reshape(-1, 2)
        np.savez(out, shade=st[rt.STATS_HEADER:].cpu().numpy().reshape(-1, 2), primary=p)


if __name__ == "__main__":
    main()
