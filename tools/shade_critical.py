"""Is the shaded C3 frame bound by its longest waves or by its total work?  The product kernel itself writes every
block's duration when the frame schedule sorts (svo_tree_schedule's cost: 100 MHz ticks), so no diagnostics instance is
needed: the frame time (HIP events) against the longest block and against the blocks' summed time over the GPU's wave
slots (7 per SIMD for the shading instances, 1024 SIMDs).  usage: python tools/shade_critical.py"""
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
    n = solid.count(d)
    rgba = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    res = {}
    for label, shadow in (("shaded", 75), ("no_shadow", 0)):
        for _ in range(12):  # (sorted after every 4th frame: the last sort's durations are read below)
            solid.shade(d, rgba, scene=scene, shadow_steps=shadow, stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            solid.shade(d, rgba, scene=scene, shadow_steps=shadow, stream=st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        _, cost = solid.schedule(rt.SCHED_SHADE, stream=st)
        dur = cost.astype(np.float64) / 100.0  # us
        slots = 7 * 1024
        res[label] = {"frame_us": round(ms * 1e3, 1), "blocks": int(len(dur)), "max_block_us": round(float(dur.max()), 1),
                      "p99_block_us": round(float(np.percentile(dur, 99)), 1), "mean_block_us": round(float(dur.mean()), 2),
                      "packed_us_7_waves": round(float(dur.sum()) / slots, 1),
                      "blocks_over_150us": int((dur > 150).sum()), "blocks_over_100us": int((dur > 100).sum())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
