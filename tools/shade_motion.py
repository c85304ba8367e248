"""The frame schedule under camera motion: shaded C3 frames (the bench scene, 1080p, S = 16384) from a camera that
turns and moves frame by frame, timed with and without the schedule (SVO_CAST_NO_SCHEDULE), interleaved.  The bench
repeats one view; a renderer's frames differ a little each time (the schedule's durations are one frame old) or, at a
cut, entirely (the schedule is then a random order of the new view's blocks).
usage: python tools/shade_motion.py [frames]"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import raytracing_test_amd as rt

    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    solid = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    scene = rt.Tree.terrain_gpu(6, 4096, 4096, 0, view=rt.VIEW_ALL)
    W, H, S = 1920, 1080, 16384
    n = W * H
    rgba = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()

    def pose(k, motion):
        if motion == "still":
            return (4.0, 90.0, 4.0), (1.0, -0.45, 1.0)
        if motion == "cut":  # a different view every frame
            yaw = math.radians(45.0 + 97.0 * k)
            return (4.0 + 37.0 * (k % 5), 90.0, 4.0 + 23.0 * (k % 3)), (math.cos(yaw), -0.45, math.sin(yaw))
        step = {"turn": 0.25, "fast": 2.0}[motion]  # degrees of yaw per frame (15 / 120 deg per second at 60 fps)
        yaw = math.radians(45.0 + step * k)
        return (4.0 + 0.1 * k, 90.0, 4.0 + 0.1 * k), (math.cos(yaw), -0.45, math.sin(yaw))

    res = {}
    for motion in ("still", "turn", "fast", "cut"):
        for flags in (0, rt.CAST_NO_SCHEDULE):
            ts = []
            with torch.cuda.stream(st):
                for k in range(-3, frames):
                    org, cam = pose(max(k, 0), motion)
                    d = solid.frame_desc(org, rt.normalize(cam), W, H, S, flags=flags)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    solid.shade(d, rgba, stream=st, scene=scene)
                    e1.record(st)
                    if k >= 0:
                        ts.append((e0, e1))
            st.synchronize()
            ms = sorted(a.elapsed_time(b) for a, b in ts)
            res["%s_%s" % (motion, "default_order" if flags else "scheduled")] = {
                "median_ms": round(ms[len(ms) // 2], 4), "mean_ms": round(sum(ms) / len(ms), 4), "max_ms": round(ms[-1], 4)}
            print(motion, "default" if flags else "scheduled", res["%s_%s" % (motion, "default_order" if flags else "scheduled")], flush=True)
    print(json.dumps({"frames": frames, "per_frame": res}), flush=True)


if __name__ == "__main__":
    main()
