#!/usr/bin/env python3
"""bench.py — primary rays/s of the gfx950 SVO raycaster on BASELINE.json's metric config.

Workload: genWorld's terrain on 4096 x 4096 columns as a depth-12
(4096^3, 6-level) tree, one 1920x1080 frame of primary rays from (4,90,4) towards
normalize(1,-0.45,1), step budget 16384, castRayFromCam semantics (every ray ends on terrain).
A "step" = one frame per GPU: with N ranks, N frames (camera poses shifted along the diagonal)
are each sharded over all ranks by interleaved 8-pixel tile rows (row r -> rank r mod N), every
rank casts its rows of every frame, and the hit records are gathered to rank 0 over RCCL.
Per-GPU work is fixed as N grows ("weak").  Inputs (tree, camera) are resident in HBM before
the timed region; the timed region is K steps between barrier + synchronize on both sides; the
reported time is the max over ranks.

Extra objects on the JSON line:
  roofline     — the cast kernel's algorithmic bytes (B_ray = 16*E_node +
                 4*E_child + B_out per ray, E from profiles/bray.json) / its average launch time,
                 measured with HIP events on the launch stream (N=1: one pair around the timed
                 region, gaps between launches included), against the 8 TB/s HBM peak;
                 traffic = HBM bytes per launch from the committed rocprofv3 PMC pass (or null).
  cpu_baseline — the oracle's C restatement of castRayFromCam + getBlock (reference layout, full
                 descent per step) timed on this host's cores on the same frame (rank 0, N=1).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
LEVELS, COLS = 6, 4096
W, H = 1920, 1080
ORIGIN = (4.0, 90.0, 4.0)
CAM = (1.0, -0.45, 1.0)
STEPS = 16384
B_OUT = 24  # hit record bytes per ray (int4 pos+steps, f32 t, u32 info)


FRAME_SHIFT = 64.0  # camera shift along the diagonal between the frames of one step (N > 1)
BRAY_KEY = {"c2": "C2_cam1_S300", "c2cam0": "C2_cam0_S300", "c3": "C3", "c5": "C5"}


def frame_origin(f):
    return (ORIGIN[0] + FRAME_SHIFT * f, ORIGIN[1], ORIGIN[2] + FRAME_SHIFT * f)


def load_bray(config="c3"):
    p = os.path.join(ROOT, "profiles", "bray.json")
    if os.path.exists(p):
        d = json.load(open(p))
        c = d.get(BRAY_KEY[config])
        if c:
            return c["e_child_per_ray"], d
    return None, None


def load_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch"), d
    return None, None


def cpu_baseline(ppx, ppy, gpu_hits=None, config="c3"):
    """Oracle (test infrastructure) timed on the host: the reference algorithm and layout."""
    from oracle import oracle as O

    O.build(native=True)
    cores = min(16, os.cpu_count() or 1)
    t0 = time.time()
    T = O.Tree.reference_world() if config.startswith("c2") else O.Tree.terrain(LEVELS, COLS, COLS, native=True, nthreads=cores)
    build_s = time.time() - t0
    dn = O.normalize(CAM)
    rng = np.random.default_rng(1)
    pix = np.sort(rng.choice(W * H, W * H // 4, replace=False))
    t0 = time.time()
    ref = T.cast_frame(ORIGIN, dn, W, H, STEPS, ppx=ppx, ppy=ppy, pixels=pix, nthreads=cores)
    dt = time.time() - t0
    one = pix[:: 64]
    t1 = time.time()
    T.cast_frame(ORIGIN, dn, W, H, STEPS, ppx=ppx, ppy=ppy, pixels=one, nthreads=1)
    dt1 = time.time() - t1
    res = {
        "value": len(pix) / dt,
        "unit": "rays/s",
        "cores": cores,
        "kind": "port",
        "sample": "%d random pixels (1/4) of the same 1080p %s frame, %d threads; oracle/oracle.c (-O3 -march=native "
                  "-ffp-contract=off) restating castRayFromCam + getBlock on the reference node/array layout" % (len(pix), config.upper(), cores),
        "single_thread_rays_per_s": len(one) / dt1,
        "tree_build_s": round(build_s, 2),
    }
    if gpu_hits is not None:
        g = gpu_hits
        res["parity_vs_gpu"] = bool(np.array_equal(g["pos"][pix], ref["pos"]) and np.array_equal(g["steps"][pix], ref["steps"]))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--config", default="c3", choices=["c2", "c2cam0", "c3", "c5"],
                    help="c3: depth-12 / 1080p (the metric); c5: depth-14 (16384^2 columns, 7 levels) / 3840x2160; c2: the "
                         "reference world (initTetraHexaTree + genWorld, 5 levels) / 1080p / S=300 from the C3 pose, c2cam0 "
                         "from the reference's default camera")
    ap.add_argument("--iterative", action="store_true", help="A/B: voxel-by-voxel DDA (SVO_CAST_ITERATIVE)")
    ap.add_argument("--stats", action="store_true", help="print traversal counters of one extra frame to stderr")
    ap.add_argument("--cast-flags", type=int, default=0, help="extra SVO_CAST_* bits (experiments)")
    ap.add_argument("--ao", type=int, default=0, help="config C4: hemisphere AO rays per primary hit (16 or 20)")
    ap.add_argument("--host-build", action="store_true", help="build the tree on the host (default: svo_build_terrain_gpu)")
    ap.add_argument("--shade", action="store_true",
                    help="SURVEY §8f.1: shaded frames (svo_shade_rays: primary + reflections + 75-step sun shadow ray), "
                         "rgba gathered instead of hit records")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal on one GPU)")
    ap.add_argument("--verify", action="store_true",
                    help="N>1: rank 0 checks the gathered, unpacked records of every frame against a one-GPU cast of it")
    ap.add_argument("--launch-events", action="store_true",
                    help="an event pair around every cast launch (default at N=1: one pair around the timed region, whose "
                         "average per launch includes the gaps between launches; per-launch pairs cost ~7 us per step)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import raytracing_test_amd as rt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)

    global LEVELS, W, H, ORIGIN, CAM, STEPS, FRAME_SHIFT
    if args.config.startswith("c2"):
        LEVELS, STEPS, FRAME_SHIFT = 5, 300, 8.0
        if args.config == "c2cam0":  # globals.cpp:20-21
            ORIGIN, CAM = (35.0, 50.0, 35.0), (1.0, 0.0, 1.0)
    if args.config == "c5":
        LEVELS, W, H = 7, 3840, 2160
        args.no_cpu_baseline = True  # the reference-format CPU tree of 16384^2 terrain exceeds its 2^32-byte pools
    if args.cols is None:
        args.cols = 4096 if args.config == "c3" else 16384
    t0 = time.time()
    if args.config.startswith("c2"):  # initTetraHexaTree + genWorld, putBlock by putBlock
        tree = rt.World.reference().build()
        build_s = time.time() - t0
        tree.upload(dev)
    elif args.host_build:
        tree = rt.Tree.terrain(LEVELS, args.cols, args.cols, nthreads=16)
        build_s = time.time() - t0
        tree.upload(dev)
    else:  # noise + build in HBM (identical arrays, tests/test_gpu_build.py); already uploaded
        tree = rt.Tree.terrain_gpu(LEVELS, args.cols, args.cols, dev)
        build_s = time.time() - t0
    info = tree.info()
    ppx, ppy = rt.proj_plane(W, H)
    cam = rt.normalize(CAM)

    from raytracing_test_amd import shard

    nframes = world
    # one launch per step covers this rank's tile rows of all N frames (each frame's shard alone
    # would fill 1/N of the GPU); records of frame f follow those of frame f-1
    origins = [frame_origin(f) for f in range(nframes)]
    desc = rt.Tree.frame_desc(origins[0], cam, W, H, STEPS, ppx, ppy, tile_row_start=rank, tile_row_step=world,
                              flags=(rt.CAST_ITERATIVE if args.iterative else 0) | args.cast_flags, ao_samples=args.ao,
                              frame_origins=origins if nframes > 1 else None)
    descs = [desc]
    gather = world > 1 and not args.no_gather
    # The exchange: frame f is displayed by rank f, so every frame's tile-row shards are gathered to
    # its own rank — one all-to-all per step (rank r sends its rows of frame f to rank f), which
    # spreads the traffic over every rank's xGMI links instead of funnelling N frames into rank 0.
    # Hit records travel as 12-B wire records (svo_hits_pack); the image (--shade) and AO counts as
    # they are.
    wire_fmt = gather and not args.shade
    n_mine = rt.Tree.count(desc) // nframes  # my records of one frame
    counts = [shard.shard_count(W, H, r, world) for r in range(world)]  # rank r's records of one frame
    nbuf = 2 if gather else 1  # the exchange of step k overlaps the cast of step k+1
    gdev = torch.device("cuda", dev)
    outs, sends, recvs = [], [], []
    for _ in range(nbuf):
        views = rt.Tree.alloc_hits(n_mine * nframes, dev, ao=args.ao > 0)
        if args.shade:  # the image is the product: exchange it instead of the hit records
            views["rgba"] = torch.zeros((n_mine * nframes, 4), dtype=torch.float32, device=gdev)
        outs.append(views)
        if gather:
            snd, rcv = [], []
            if wire_fmt:
                snd.append(torch.zeros((n_mine * nframes, rt.WIRE_BYTES), dtype=torch.uint8, device=gdev))
                rcv.append(torch.zeros((W * H, rt.WIRE_BYTES), dtype=torch.uint8, device=gdev))
            if args.ao:
                snd.append(views["ao"])
                rcv.append(torch.zeros(W * H, dtype=torch.uint8, device=gdev))
            if args.shade:
                snd.append(views["rgba"])
                rcv.append(torch.zeros((W * H, 4), dtype=torch.float32, device=gdev))
            sends.append(snd)
            recvs.append(rcv)
    stream = torch.cuda.Stream(device=dev)
    src_descs, frame_hits = None, None
    if wire_fmt:  # my frame (rank) from every rank's rows, unpacked into one record buffer
        src_descs = [rt.Tree.frame_desc(origins[rank], cam, W, H, STEPS, ppx, ppy, tile_row_start=r, tile_row_step=world)
                     for r in range(world)]
        frame_hits = rt.Tree.alloc_hits(W * H, dev)
    offs = np.concatenate([[0], np.cumsum(counts)]).tolist()
    pending = {}  # step -> (async all-to-all works, send buffers kept alive)

    def unpack_step(k):
        """wait (nccl: on the stream) for the exchange of step k, then unpack my frame's records"""
        works, _ = pending.pop(k)
        for w in works:
            w.wait()
        b = k % nbuf
        if args.dist_backend != "nccl":  # gloo rehearsal: received on the host
            for i, h in enumerate(recv_host[b]):
                recvs[b][i].copy_(h)
        if wire_fmt:
            for r in range(world):
                part = {key: v[offs[r]:offs[r + 1]] for key, v in frame_hits.items()}
                tree.unpack_hits(src_descs[r], recvs[b][0][offs[r]:offs[r + 1]], part, stream)

    recv_host = None
    if gather and args.dist_backend != "nccl":
        recv_host = [[torch.empty_like(x, device="cpu") for x in rcv] for rcv in recvs]

    def one_step(k, events=None):
        b = k % nbuf
        with torch.cuda.stream(stream):
            if events is not None:
                events[0][0].record(stream)
            if args.shade:
                tree.shade(desc, outs[b]["rgba"], out=outs[b], stream=stream)
            else:
                tree.cast(desc, outs[b], stream)
            if events is not None:
                events[0][1].record(stream)
            if not gather:
                return
            if wire_fmt:
                tree.pack_hits(desc, outs[b], sends[b][0], stream)
            # asynchronous: the next step's cast runs while RCCL moves this one over xGMI (gloo
            # rehearsal: the same pipeline through host copies); the unpack of step k-1 follows
            works, keep = [], []
            for i, (snd, rcv) in enumerate(zip(sends[b], recvs[b])):
                src = snd if args.dist_backend == "nccl" else snd.cpu()
                dst = rcv if args.dist_backend == "nccl" else recv_host[b][i]
                works.append(dist.all_to_all_single(dst, src, output_split_sizes=counts, input_split_sizes=[n_mine] * world,
                                                    async_op=True))
                keep.append(src)
            pending[k] = (works, keep)
            if (k - 1) in pending:
                unpack_step(k - 1)

    def drain():
        with torch.cuda.stream(stream):
            for k in sorted(pending):
                unpack_step(k)

    step_no = 0
    for _ in range(args.warmup):
        one_step(step_no)
        step_no += 1
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]] for _ in range(args.steps)]
    reg = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    # at N=1 the launches run back to back on one stream: one event pair around the timed region
    # gives their average (gaps included); with a gather in between, pairs around each launch
    args.region_events = world == 1 and not args.launch_events
    t0 = time.perf_counter()
    if args.region_events:
        reg[0].record(stream)
    for k in range(args.steps):
        one_step(step_no, None if args.region_events else evs[k])
        step_no += 1
    if args.region_events:
        reg[1].record(stream)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if args.region_events:  # launches back to back on one stream (no gather in between at N=1)
        kern_ms = [reg[0].elapsed_time(reg[1]) / args.steps]
    else:
        kern_ms = [e[0].elapsed_time(e[1]) for step in evs for e in step]
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_rays = W * H * nframes * args.steps  # every rank's share of every frame, all steps
    value = total_rays / elapsed
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    rays_per_launch = rt.Tree.count(descs[0])
    verified = None
    if args.verify and wire_fmt:
        # my frame reassembled from every rank's unpacked records == a one-GPU cast of it
        torch.cuda.synchronize()
        one = rt.decode_hits(tree.cast_frame(origins[rank], cam, W, H, STEPS, ppx, ppy, flags=args.cast_flags))
        got = rt.decode_hits(frame_hits)
        ok = True
        for r in range(world):
            rows = shard.shard_pixel_rows(H, r, world)
            idx = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
            ok &= all(np.array_equal(got[key][offs[r]:offs[r + 1]], one[key][idx]) for key in ("pos", "steps", "hit", "axis", "material", "t"))
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        verified = bool(flag.item())

    if args.stats and rank == 0:
        d0 = descs[0]
        nblk = rt.Tree.blocks(d0)
        for mode in (rt.CAST_STATS, rt.CAST_TIMELINE):
            st = torch.zeros(rt.STATS_HEADER + 2 * nblk + rt.Tree.count(d0), dtype=torch.int64, device=dev)
            d0.flags |= mode
            d0.stats = st.data_ptr()
            tree.cast(d0, outs[0], stream)
            torch.cuda.synchronize()
            d0.flags &= ~mode
            allv = st.cpu().numpy()
            if mode == rt.CAST_STATS:
                vals = allv[:rt.STATS_HEADER]
                if os.environ.get("SVO_RAY_WORK"):  # per-pixel lookups / brick steps for offline analysis
                    np.save(os.environ["SVO_RAY_WORK"], allv[rt.STATS_HEADER + 2 * nblk:])
                per = [v / max(1, vals[0]) * (64 if k.startswith("wave_") and not k.endswith("_x64") else 1) for k, v in zip(rt.STAT_NAMES, vals)]
                print("stats per ray (wave_* per wave): " + ", ".join("%s=%.3f" % (k, v) for k, v in zip(rt.STAT_NAMES, per)) +
                      "; SIMD efficiency %.3f" % (vals[7] / max(1, vals[8])), file=sys.stderr)
                continue
            stamps = allv[rt.STATS_HEADER:rt.STATS_HEADER + 2 * nblk].reshape(-1, 2)
            stamps = stamps[stamps[:, 1] > 0].astype(np.float64) / 100.0  # launched blocks; us (100 MHz)
            t0s = stamps[:, 0].min()
            dur = stamps[:, 1] - stamps[:, 0]
            span = stamps[:, 1].max() - t0s
            bins = np.linspace(0, span, 17)
            res = [int(((stamps[:, 0] - t0s < b1) & (stamps[:, 1] - t0s > b0)).sum()) for b0, b1 in zip(bins[:-1], bins[1:])]
            tenths = [float(np.mean(c)) for c in np.array_split(dur, 10)]
            ends = np.sort(stamps[:, 1] - t0s)
            print("timeline: span %.1f us, mean block %.1f us, max %.1f us, last 10%% of blocks end after %.1f us; blocks overlapping "
                  "each 1/16 of the span %s; mean block us per tenth of the grid %s"
                  % (span, dur.mean(), dur.max(), ends[int(len(ends) * 0.9)], res, ["%.0f" % x for x in tenths]), file=sys.stderr)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    e_child, bray_meta = load_bray(args.config)
    roof = None
    if e_child is not None:
        b_ray = 16.0 * (e_child + 1.0) + 4.0 * e_child + B_OUT
        achieved = b_ray * rays_per_launch / avg_kernel_s / 1e9
        traffic, _ = load_traffic() if args.config == "c3" else (None, None)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "bytes_per_ray": round(b_ray, 2), "avg_launch_ms": round(avg_kernel_s * 1e3, 4)}
    cpu = None
    if args.shade:
        roof = None  # the roofline model (§8d) prices primary traversal only
    if world == 1 and not args.no_cpu_baseline and not args.ao and not args.shade:
        hits = rt.decode_hits(outs[0])
        cpu = cpu_baseline(ppx, ppy, hits, args.config)
    line = {
        "metric": ("shaded primary rays/sec (reflections + sun shadow ray)" if args.shade else
                   {"c2": "primary rays/sec at 1080p, reference-world SVO (config 2); achieved HBM GB/s vs roofline",
                    "c2cam0": "primary rays/sec at 1080p, reference-world SVO (config 2); achieved HBM GB/s vs roofline",
                    "c3": "primary rays/sec at 1080p, depth-12 SVO; achieved HBM GB/s vs roofline",
                    "c5": "primary rays/sec at 4K, depth-14 SVO; achieved HBM GB/s vs roofline"}[args.config]),
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: the reference world (initTetraHexaTree + genWorld on 200x200 columns), built in-process"
                 if args.config.startswith("c2") else
                 "synthetic: genWorld OpenSimplex terrain (seeds 42/64/100) on %dx%d columns, built in-process" % (args.cols, args.cols)),
        "config": {"ao_samples": args.ao, "shade": args.shade,
                   "workload": ("C4 (C3 + %d hemisphere AO rays per hit, 5 steps each): " % args.ao if args.ao else "") +
                   ("shaded (low_res.frag colour model, 75-step shadow rays): " if args.shade else "") +
                   {"c2": "C2: the reference world (5 levels, 1024^3), 1920x1080",
                    "c2cam0": "C2: the reference world (5 levels, 1024^3), 1920x1080",
                    "c3": "C3: depth-12 SVO (%d^2 terrain columns, 6 levels, 4096^3), 1920x1080" % args.cols,
                    "c5": "C5: depth-14 SVO (%d^2 terrain columns, 7 levels, 16384^3), 3840x2160" % args.cols}[args.config] +
                   " primary rays per GPU per step, camera (%g,%g,%g)->normalize(%g,%g,%g), S=%d, castRayFromCam semantics"
                   % (ORIGIN + CAM + (STEPS,)),
                   "frames_per_step": nframes, "rays_per_step": W * H * nframes, "parallelism": "tile-row shard x%d" % world,
                   "launches_per_step": 1, "gather": gather,
                   "exchange": ("frame f gathered to rank f (one all-to-all per step, overlapped with the next cast): " +
                                ("rgba image" if args.shade else "12-B wire hit records (svo_hits_pack), unpacked on arrival" +
                                 (" + AO counts" if args.ao else ""))) if gather else None, "tree_nodes": info.n_nodes,
                   "tree_bytes": info.n_nodes * 16 + info.n_mat_bytes, "tree_build_s": round(build_s, 3),
                   "tree_builder": "host" if args.host_build else "gpu"},
        "roofline": roof,
        "cpu_baseline": cpu,
        **({"gather_verified": verified} if verified is not None else {}),
        "launch_timing": "one HIP event pair around the timed region on the launch stream (average per launch, gaps "
                         "included)" if args.region_events else "a HIP event pair around every launch on its stream",
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
