"""Where the C5 strong-scaling exchange spends its time, measured on one GPU:
the cast of a whole 4K frame and of a 1/8 shard, svo_hits_pack of each, svo_hits_unpack of a whole
frame, the one-rank RCCL exchange (pack + self-send + scatter-unpack) and a plain device copy of the
same wire bytes.  HIP events on one stream, median of --reps repetitions.
usage: python tools/xchg_parts.py [--config c5|c3] [--reps 20]"""
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
    ap.add_argument("--shards", type=int, default=8)
    a = ap.parse_args()
    import torch

    import raytracing_test_amd as rt

    cfg = {"c5": (7, 16384, 3840, 2160), "c3": (6, 4096, 1920, 1080)}[a.config]
    levels, cols, W, H = cfg
    tree = rt.Tree.terrain_gpu(levels, cols, cols, 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    org = (4.0, 90.0, 4.0)
    N = a.shards
    full = rt.Tree.frame_desc(org, cam, W, H, 16384)
    shard = rt.Tree.frame_desc(org, cam, W, H, 16384, tile_row_start=0, tile_row_step=N)
    nf, ns = rt.Tree.count(full), rt.Tree.count(shard)
    of, osh = rt.Tree.alloc_hits(nf, 0), rt.Tree.alloc_hits(ns, 0)
    back = rt.Tree.alloc_hits(nf, 0)
    wf = torch.empty((nf, rt.WIRE_BYTES), dtype=torch.uint8, device="cuda")
    ws = torch.empty((ns, rt.WIRE_BYTES), dtype=torch.uint8, device="cuda")
    wcopy = torch.empty_like(wf)
    x = rt.Exchange(1, 0, rt.Exchange.unique_id(), 0)
    frames_out = rt.Tree.alloc_hits(nf, 0)
    s = torch.cuda.current_stream()

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return round(statistics.median(ms) * 1e3, 1)  # us

    res = {"config": a.config, "rays_full": nf, "rays_shard": ns, "shards": N, "wire_bytes_per_ray": rt.WIRE_BYTES}
    res["cast_full_us"] = timed(lambda: tree.cast(full, of, s))
    res["cast_shard_us"] = timed(lambda: tree.cast(shard, osh, s))
    res["pack_full_us"] = timed(lambda: tree.pack_hits(full, of, wf, s))
    res["pack_shard_us"] = timed(lambda: tree.pack_hits(shard, osh, ws, s))
    res["unpack_full_us"] = timed(lambda: tree.unpack_hits(full, wf, back, s))
    res["copy_wire_full_us"] = timed(lambda: wcopy.copy_(wf))
    res["exchange_1rank_us"] = timed(lambda: x.frames(tree, full, of, frames_out, s))
    # the fused path (svo_cast_wire + svo_exchange_wire / svo_wire_scatter): wire records from the cast kernel
    wbf, wbs = tree.wire_bytes(full), tree.wire_bytes(shard)
    res["compact_wire_bytes"] = wbf
    cwf = torch.empty((nf, wbf), dtype=torch.uint8, device="cuda")
    cws = torch.empty((ns, wbs), dtype=torch.uint8, device="cuda")
    res["cast_wire_full_us"] = timed(lambda: tree.cast_wire(full, cwf, None, s))
    res["cast_wire_shard_us"] = timed(lambda: tree.cast_wire(shard, cws, None, s))
    res["scatter_shard_us"] = timed(lambda: tree.wire_scatter(shard, cws, frames_out, None, s))
    res["exchange_wire_1rank_us"] = timed(lambda: x.wire(tree, full, cwf, frames_out, None, s))
    res["copy_compact_full_us"] = timed(lambda: cwf[: nf // 2].copy_(cwf[nf // 2: 2 * (nf // 2)]))
    torch.cuda.synchronize()
    tree.cast(full, of, s)
    tree.cast_wire(full, cwf, None, s)
    x.wire(tree, full, cwf, frames_out, None, s)
    torch.cuda.synchronize()
    ok = all(torch.equal(back[k], of[k]) for k in of) and all(torch.equal(frames_out[k], of[k]) for k in of)
    res["roundtrip_equal"] = ok
    x.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
