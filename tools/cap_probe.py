"""Launch-tail probe (round 3): with a library built with -D SVO_ITER_CAP=M (diagnostics), rays still running after
M traversal iterations stop and report steps_left -1.  Prints the C3 launch time and how many rays were cut (the
work a continuation pass would take over).  usage: SVO_LIB=variants/libsvo_capM.so python tools/cap_probe.py"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import raytracing_test_amd as rt

    reps = int(os.environ.get("REPS", "20"))
    tree = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    d = rt.Tree.frame_desc((4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0)), 1920, 1080, 16384)
    out = rt.Tree.alloc_hits(rt.Tree.count(d), 0)
    s = torch.cuda.current_stream()
    for _ in range(3):
        tree.cast(d, out, s)
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        tree.cast(d, out, s)
        e1.record(s)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    cut = (out["pos_steps"][:, 3] == -1)
    n = int(cut.sum().item())
    # cut rays per 64-ray wave (16x4 footprints, dispatch order = record order of 8-row tile rows)
    print(json.dumps({"lib": os.path.basename(os.environ.get("SVO_LIB", "default")), "us": round(statistics.median(ms) * 1e3, 1),
                      "cut_rays": n, "cut_frac": round(n / cut.numel(), 5)}), flush=True)


if __name__ == "__main__":
    main()
