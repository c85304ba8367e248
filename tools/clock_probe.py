"""Clock probe (round 5): is the far-field waves' slow-down in a full frame (top 4 tile rows alone: ~140 us; inside the
frame: ~170 us) a lower shader clock or more cycles?  Needs the diagnostic build of tools/variants/clock_probe.patch
(SVO_LIB=variants/libsvo_clock.so): the TIMELINE instance then also stores each block's s_memtime (shader clock) at
start and end after the stamps.  Per launch it prints the block durations (us), cycles and the clock (cycles / duration)
of all blocks and of the 100 longest.  usage: SVO_LIB=... python tools/clock_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import raytracing_test_amd as rt

    W, H, S = 1920, 1080, 16384
    tree = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    org = (4.0, 90.0, 4.0)
    rows = H // 8
    res = {}
    for name, start, step in (("full", 0, 1), ("top4", rows - 4, 1), ("top34", rows - 34, 1)):
        d = rt.Tree.frame_desc(org, cam, W, H, S, tile_row_start=start, tile_row_step=step, flags=rt.CAST_TIMELINE)
        nb = rt.Tree.blocks(d)
        out = rt.Tree.alloc_hits(rt.Tree.count(d), 0)
        st = torch.zeros(rt.STATS_HEADER + 4 * nb, dtype=torch.int64, device="cuda")
        d.stats = st.data_ptr()
        for _ in range(3):  # (warm: the last launch's stamps are read)
            tree.cast(d, out)
        torch.cuda.synchronize()
        v = st.cpu().numpy()
        rt_ = v[rt.STATS_HEADER:rt.STATS_HEADER + 2 * nb].reshape(-1, 2).astype(np.float64)
        cy = v[rt.STATS_HEADER + 2 * nb:rt.STATS_HEADER + 4 * nb].reshape(-1, 2).astype(np.float64)
        dur_us = (rt_[:, 1] - rt_[:, 0]) / 100.0
        cyc = cy[:, 1] - cy[:, 0]
        ghz = cyc / (dur_us * 1e3)
        top = np.argsort(dur_us)[::-1][:100]
        res[name] = {"blocks": nb, "span_us": round((rt_[:, 1].max() - rt_[:, 0].min()) / 100.0, 1),
                     "mean_us": round(dur_us.mean(), 2), "mean_ghz": round(float(np.median(ghz)), 3),
                     "top100_us": round(dur_us[top].mean(), 1), "top100_mcycles": round(cyc[top].mean() / 1e6, 4),
                     "top100_ghz": round(float(np.median(ghz[top])), 3), "max_us": round(dur_us.max(), 1)}
        if name == "full":  # the top 4 tile rows' blocks (dispatched first) inside the whole frame
            k = 4 * (nb // rows)
            tk = np.argsort(dur_us[:k])[::-1][:100]
            res["full_top4rows"] = {"blocks": k, "mean_us": round(dur_us[:k].mean(), 2), "mean_mcycles": round(cyc[:k].mean() / 1e6, 4),
                                    "mean_ghz": round(float(np.median(ghz[:k])), 3), "top100_us": round(dur_us[:k][tk].mean(), 1),
                                    "top100_mcycles": round(cyc[:k][tk].mean() / 1e6, 4)}
        if name == "top4":
            res["top4"]["mean_mcycles"] = round(cyc.mean() / 1e6, 4)
        print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
