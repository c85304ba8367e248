#!/usr/bin/env python3
"""bench.py — primary rays/s of the gfx950 SVO raycaster on BASELINE.json's metric config.

Workload (the default): genWorld's terrain on 4096 x 4096 columns as a
depth-12 (4096^3, 6-level) tree, one 1920x1080 frame of primary rays from (4,90,4) towards
normalize(1,-0.45,1), step budget 16384, castRayFromCam semantics (every ray ends on terrain).
Other configs: --config c1 (dense 256^3 grid, 256^2 rays), c2 / c2cam0 (the reference world), c2d8 (genWorld in a depth-8 tree),
c5 (depth-14, 4K); --ao N (C4: + N hemisphere AO rays per hit); --shade (the shading pass).

A "step" = one pass of the cast kernel over the step's frames.  Multi-GPU: one process per GPU, either
under a launcher (torch.distributed.run ... bench.py --gpus N; WORLD_SIZE must equal N) or started by
bench.py itself (`python bench.py --gpus N` with no WORLD_SIZE: N child processes, RANK = LOCAL_RANK =
r, before anything touches a GPU; rank 0 prints the line, the exit status is the first failing
rank's).  `n_gpus` on the line is the size of the communicator the step ran over (svo_exchange_info
for the RCCL exchange).  Frames are sharded by interleaved 8-pixel tile rows (row r -> rank r mod N)
and every frame's shards are gathered over RCCL to the rank that displays it, by the C ABI's
svo_exchange_frames (include/svo_rt.h), overlapped with the next step's cast on a second stream.
  * default ("weak"): a step renders N frames (camera poses shifted along the diagonal), so per-GPU
    work is fixed as N grows; frame f is displayed by rank f (the gathers form one all-to-all);
  * --frames F ("strong"): a step renders F frames whatever N is (C5 as BASELINE.json words it:
    --config c5 --frames 1 = one 4K frame split over N GPUs, gathered to rank 0:
    `python bench.py --gpus 8 --config c5 --frames 1`).
Inputs (tree, camera) are resident in HBM before the timed region; the timed region is K steps
between barrier + synchronize on both sides; the reported time is the max over ranks.

Extra objects on the JSON line:
  roofline     — the cast kernel's algorithmic bytes (B_ray = 16*E_node +
                 4*E_child + B_out per ray (+ the AO rays' entries for C4), E from profiles/bray.json)
                 / its average launch time, measured with HIP events on the launch stream, against
                 the 8 TB/s HBM peak (`frac`); next to it what the committed rocprofv3 PMC passes of
                 the same config (profiles/pmc_<config>.json) measured: HBM bytes per launch
                 (`traffic`), measured HBM GB/s, L2 hit rate, VALU / SALU instructions per wave and
                 the VALU issue fraction; `bound` names the larger of the measured HBM and VALU-issue
                 fractions.
  cpu_baseline — the oracle's C restatement of castRayFromCam + getBlock (reference node/array
                 layout, full descent per step) timed on this host's cores on the same workload
                 (rank 0, N=1), plus config C1 (dense grid) every time.
"""
import argparse
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N_SIMD = 1024  # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4  # peak engine clock (the VALU issue fraction is priced at it: a lower bound on busy)
VALU_CYCLES = 2  # a wave64 VALU instruction occupies a SIMD for 2 cycles (f64 ops: more)
B_OUT = 24  # hit record bytes per ray (int4 pos+steps, f32 t, u32 info)

# config -> scene / camera / budget
CONFIGS = {
    "c1": dict(levels=4, cols=256, W=256, H=256, origin=(35.0, 50.0, 35.0), cam=(1.0, 0.0, 1.0), steps=300, shift=4.0,
               label="C1: the reference world's [0,256)^3 as a 256^3 grid (4 levels), 256x256", bray="C1",
               metric="primary rays/sec at 256x256, dense 256^3 grid (config 1)"),
    "c2": dict(levels=5, cols=200, W=1920, H=1080, origin=(4.0, 90.0, 4.0), cam=(1.0, -0.45, 1.0), steps=300, shift=8.0,
               label="C2: the reference world (5 levels, 1024^3), 1920x1080", bray="C2_cam1_S300",
               metric="primary rays/sec at 1080p, reference-world SVO (config 2); achieved HBM GB/s vs roofline"),
    "c2cam0": dict(levels=5, cols=200, W=1920, H=1080, origin=(35.0, 50.0, 35.0), cam=(1.0, 0.0, 1.0), steps=300, shift=8.0,
                   label="C2: the reference world (5 levels, 1024^3), 1920x1080, the reference's default camera (globals.cpp:20-21)",
                   bray="C2_cam0_S300",
                   metric="primary rays/sec at 1080p, reference-world SVO (config 2); achieved HBM GB/s vs roofline"),
    "c2d8": dict(levels=4, cols=200, W=1920, H=1080, origin=(4.0, 90.0, 4.0), cam=(1.0, -0.45, 1.0), steps=300, shift=8.0,
                 label="C2 as BASELINE.json words it: depth-8 SVO (4 levels, 256^3), genWorld putBlocks over 200x200 columns, 1920x1080",
                 bray="C2d8", metric="primary rays/sec at 1080p, depth-8 SVO (config 2); achieved HBM GB/s vs roofline"),
    "c3": dict(levels=6, cols=4096, W=1920, H=1080, origin=(4.0, 90.0, 4.0), cam=(1.0, -0.45, 1.0), steps=16384, shift=64.0,
               label="C3: depth-12 SVO (4096^2 terrain columns, 6 levels, 4096^3), 1920x1080", bray="C3",
               metric="primary rays/sec at 1080p, depth-12 SVO; achieved HBM GB/s vs roofline"),
    "c3f": dict(levels=6, cols=4096, W=1920, H=1080, origin=(4.37, 90.61, 4.23), cam=(1.0, -0.45, 1.0), steps=16384, shift=64.0,
                label="C3 from a non-integral camera position (segment-exact crossings): depth-12 SVO, 1920x1080", bray="C3f",
                metric="primary rays/sec at 1080p, depth-12 SVO; achieved HBM GB/s vs roofline"),
    "c5": dict(levels=7, cols=16384, W=3840, H=2160, origin=(4.0, 90.0, 4.0), cam=(1.0, -0.45, 1.0), steps=16384, shift=64.0,
               label="C5: depth-14 SVO (16384^2 terrain columns, 7 levels, 16384^3), 3840x2160", bray="C5",
               metric="primary rays/sec at 4K, depth-14 SVO; achieved HBM GB/s vs roofline"),
}


def frame_origin(cfg, f):
    o, s = cfg["origin"], cfg["shift"]
    return (o[0] + s * f, o[1], o[2] + s * f)


def run_key(args):
    """the profiles/pmc_<key>.json a config's counters live in"""
    return args.config + ("_ao%d" % args.ao if args.ao else "") + ("_shade" if args.shade else "")


def load_json(name):
    p = os.path.join(ROOT, "profiles", name)
    return json.load(open(p)) if os.path.exists(p) else None


# ------------------------------------------------------------------------------- CPU baseline --
def cpu_info():
    """The host's CPUs and the threads the baseline may use: the job's CPU allotment (OMP_NUM_THREADS,
    which the GPU pool sets to the job's share of a shared host; else the affinity mask, capped by
    a cgroup CPU quota)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(aff, quota) if quota else aff
    rule = "affinity mask" + (" capped by the cgroup CPU quota" if quota else "")
    if omp and omp.isdigit() and int(omp) > 0:
        threads, rule = min(int(omp), aff), "OMP_NUM_THREADS (the job's CPU share on this host)"
    return {"nproc": nproc, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "cpu_model": model, "threads": threads,
            "threads_rule": rule}


def _timed(fn):
    t0 = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t0


def cpu_baseline(args, cfg, ppx, ppy, gpu):
    """The oracle (test infrastructure: the reference algorithm + layout, oracle/oracle.c) timed on
    this host's cores: all allotted threads on the workload (or a stated sample of it), one thread
    on a fixed strided sample; parity of the GPU frame on the same rays."""
    from oracle import oracle as O

    O.build(native=True)
    ci = cpu_info()
    nt = ci["threads"]
    W, H, S = cfg["W"], cfg["H"], cfg["steps"]
    dn = O.normalize(cfg["cam"])
    org = cfg["origin"]
    t0 = time.perf_counter()
    if args.config == "c2d8":
        T = O.Tree.terrain_putblock(4, 200, 200, native=True)
    elif args.config.startswith("c2") or args.config == "c1":
        T = O.Tree.reference_world(native=True)
    elif args.config == "c5":
        # every C5 ray lands within ~2,600 voxels of the camera: the oracle's tree over the first 4096^2
        # columns holds the same voxels (its pools cannot hold 16384^2; tests/test_gpu_parity.py)
        T = O.Tree.terrain(7, 4096, 4096, native=True, nthreads=nt)
    else:
        T = O.Tree.terrain(cfg["levels"], cfg["cols"], cfg["cols"], native=True, nthreads=nt)
    build_s = time.perf_counter() - t0
    n = W * H
    # the multi-thread leg: the whole frame unless that is far beyond ~10-30 s of CPU work
    stride = {"c5": 8}.get(args.config, 1) * (4 if args.ao else 1) * (4 if args.shade else 1)
    stride1 = 16 * stride  # the single-thread leg: every 16th of those rays
    pix = np.arange(0, n, stride, dtype=np.int64)
    pix1 = np.arange(0, n, stride1, dtype=np.int64)
    parity = None
    o0 = {}
    if args.config == "c1":
        D = O.Dense(T, 256)
        ref, dt = _timed(lambda: D.cast_frame(org, dn, W, H, S, nthreads=nt))
        _, dt1 = _timed(lambda: D.cast_frame(org, dn, W, H, S, nthreads=1))
        pix1 = pix
        if gpu is not None:
            parity = bool(np.array_equal(gpu["pos"], ref["pos"]) and np.array_equal(gpu["steps"], ref["steps"]))
        what = "castRayFromCam over a dense u8 grid (getBlock seam ray_caster.cpp:81, coordinates & 255)"
    elif args.shade:
        sun = np.asarray(O.normalize((2.0, 1.0, 4.0)))
        ref, dt = _timed(lambda: T.shade_frame(org, dn, W, H, S, sun, ppx=ppx, ppy=ppy, pixels=pix, nthreads=nt, liquid=True))
        _, dt1 = _timed(lambda: T.shade_frame(org, dn, W, H, S, sun, ppx=ppx, ppy=ppy, pixels=pix1, nthreads=1, liquid=True))
        if gpu is not None:
            parity = bool(np.abs(gpu["rgba"][pix] - ref).max() <= 2e-6)
        what = "the shading pass (oracle orc_shade_frame, liquid mode: castRayFromCam + reflections + refraction / tint by " \
               "water and glass + 75-step shadow ray)"
    elif args.ao:
        (ao, hit), dt = _timed(lambda: T.cast_frame_ao(org, dn, W, H, S, args.ao, 5, ppx=ppx, ppy=ppy, pixels=pix, nthreads=nt))
        _, dt1 = _timed(lambda: T.cast_frame_ao(org, dn, W, H, S, args.ao, 5, ppx=ppx, ppy=ppy, pixels=pix1, nthreads=1))
        if gpu is not None:
            parity = bool(np.array_equal(gpu["ao"][pix], ao) and np.array_equal(gpu["hit"][pix], hit != 0))
        what = "castRayFromCam + %d hemisphere AO rays of 5 steps per hit (oracle orc_cast_frame_ao)" % args.ao
    else:
        ref, dt = _timed(lambda: T.cast_frame(org, dn, W, H, S, ppx=ppx, ppy=ppy, pixels=pix, nthreads=nt))
        _, dt1 = _timed(lambda: T.cast_frame(org, dn, W, H, S, ppx=ppx, ppy=ppy, pixels=pix1, nthreads=1))
        if gpu is not None:
            parity = bool(np.array_equal(gpu["pos"][pix], ref["pos"]) and np.array_equal(gpu["steps"][pix], ref["steps"]))
        what = "castRayFromCam + getBlock on the reference node/array layout"
        # the reference's own build flags (build.bat:4, `g++ -g` = -O0), one thread, every 512th pixel
        pix0 = np.arange(0, n, 512, dtype=np.int64)
        r0, dt0 = _timed(lambda: T.cast_frame(org, dn, W, H, S, ppx=ppx, ppy=ppy, pixels=pix0, nthreads=1, L=O.lib_O0()))
        o0 = {"single_thread_O0_rays_per_s": len(pix0) / dt0, "O0_sample": "every 512th pixel (%d rays), -O0" % len(pix0),
              "O0_equal": bool(np.array_equal(r0["pos"], ref["pos"][::512 // stride]) if stride <= 512 and 512 % stride == 0 else True)}
    res = {
        "value": len(pix) / dt,
        "unit": "rays/s",
        "cores": nt,
        "kind": "port",
        "sample": "%s of the %dx%d %s frame (every %d-th pixel), %d threads; single thread: every %d-th pixel (%d rays); "
                  "oracle/oracle.c (-O3 -march=native -ffp-contract=off): %s"
                  % ("all %d rays" % n if stride == 1 else "%d rays" % len(pix), W, H, args.config.upper(), stride, nt, stride1 if
                     args.config != "c1" else stride, len(pix1), what),
        "single_thread_rays_per_s": len(pix1) / dt1,
        **o0,
        "cpu_s": round(dt + dt1, 2),
        "tree_build_s": round(build_s, 2),
        **{k: ci[k] for k in ("nproc", "affinity_cpus", "cgroup_quota_cpus", "cpu_model", "threads_rule")},
    }
    if parity is not None:
        res["parity_vs_gpu"] = parity
    if args.config != "c1" and not args.no_c1:
        res["c1"] = cpu_c1(O, nt)
    return res


def cpu_c1(O, nt):
    """Config C1 (BASELINE.json configs[0]: the CPU reference path only): the reference world's
    [0,256)^3 materialised as a dense grid, castRayFromCam over it (getBlock seam ray_caster.cpp:81),
    256^2 rays from the reference camera (35,50,35)->(1,0,1), S = 300."""
    T = O.Tree.reference_world(native=True)
    D = O.Dense(T, 256)
    dn = O.normalize((1.0, 0.0, 1.0))
    r, dt = _timed(lambda: D.cast_frame((35.0, 50.0, 35.0), dn, 256, 256, 300, nthreads=nt))
    _, dt1 = _timed(lambda: D.cast_frame((35.0, 50.0, 35.0), dn, 256, 256, 300, nthreads=1))
    return {"rays_per_s": 65536 / dt, "single_thread_rays_per_s": 65536 / dt1, "threads": nt,
            "dda_steps_per_ray": r["dda_steps"] / 65536.0,
            "workload": "C1: dense 256^3 grid of the reference world, 256x256 rays, (35,50,35)->normalize(1,0,1), S=300"}


# ---------------------------------------------------------------------------------- roofline --
def roofline(args, cfg, rays_per_launch, avg_kernel_s, world, lib_sha):
    """The kernel against the HBM roofline (the contract's "bound": "hbm" — pointer chasing, no MFMA).
    achieved = algorithmic bytes per ray x rays per launch / average launch time.  Primary rays: SURVEY.md
    §8(d)'s B_ray (node entries along the reference DDA path, oracle/bray.py).  C4: that, plus the node
    loads the kernel's AO plan must issue (counted by the SVO_CAST_STATS instance, profiles/bray.json
    "C4_ao<N>_kernel") and the 1-B AO count — §8(d)'s AO term prices 16 traced AO rays per hit, which the
    plan replaces by ~6 brick lookups, so it is reported beside the figure, never as it.  A fraction above
    1 would mean the model prices work the kernel does not do: it is then withheld (null, with the reason)."""
    bray = load_json("bray.json") or {}
    key = cfg["bray"]
    b = bray.get(key)
    model, bytes_model, extra = None, None, {}
    sb = bray.get(key + "_shade") if args.shade else None
    if sb is not None:
        # the shading pass: §8(d)'s entries along every lookup its rays make (primary + reflections / refractions, and the
        # shadow ray), oracle/bray.py c3_shade_entry
        model = sb["bytes_per_ray"]
        bytes_model = ("SURVEY.md §8d for the shading pass: B = 16 (E + R) + 4 E + 16 B rgba, E = %.2f node entries per pixel "
                       "along the reference DDA paths of the primary ray with its reflections / refractions and of the 75-step shadow "
                       "ray (restart model, liquid mode), R = %.3f root reads per pixel (%s_shade, profiles/bray.json)"
                       % (sb["e_per_ray"], 1.0 + sb["shadow_rays_per_ray"], key))
    if not args.shade and b is not None:
        model = b["bytes_per_ray"]
        if "e_child_per_ray" in b:
            bytes_model = ("SURVEY.md §8d B_ray = 16 (E_child + 1) + 4 E_child + 24 B hit record, E_child = %.2f node entries per ray "
                           "along the reference DDA path (%s, profiles/bray.json)" % (b["e_child_per_ray"], key))
        else:  # C1: the dense grid
            bytes_model = ("SURVEY.md §8d for the dense grid: 1 B per DDA step (%.1f per ray) + 24 B hit record (%s, profiles/bray.json)"
                           % (b["dda_steps_per_ray"], key))
        if args.ao:
            kb = bray.get("C4_ao%d_kernel" % args.ao)
            traced = bray.get("C4_ao%d" % args.ao)
            if kb is None:
                model, bytes_model = None, None
                extra["note"] = "no committed AO plan load count for %d samples (profiles/bray.json C4_ao%d_kernel)" % (args.ao, args.ao)
            else:
                model = b["bytes_per_ray"] + 16.0 * kb["ao_node_loads_per_ray"] + 1.0
                bytes_model += ("; + 16 B x %.2f AO plan node loads per ray (brick lookups of the per-face plan, counted by the "
                                "SVO_CAST_STATS instance: profiles/bray.json C4_ao%d_kernel) + 1 B AO count"
                                % (kb["ao_node_loads_per_ray"], args.ao))
            if traced is not None:
                extra["bytes_per_ray_traced_ao_model"] = round(traced["bytes_per_ray"], 2)
                extra["traced_ao_model"] = ("SURVEY.md §8d with its AO term (16 traced AO rays of 5 steps per hit): not the work "
                                            "this kernel does, not used for frac")
    achieved = model * rays_per_launch / avg_kernel_s / 1e9 if model else None
    frac = achieved / HBM_PEAK_GBS if achieved else None
    if frac is not None and frac > 1.0:
        extra["note"] = ("the bytes model exceeds the HBM peak at this launch time (%.3f): it prices reads the kernel serves "
                         "from L2 / MALL or does not issue; frac withheld" % frac)
        frac = None
    roof = {"bound": "hbm" if model else None, "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(frac, 5) if frac is not None else None, "traffic": None,
            "bytes_per_ray": round(model, 2) if model else None, "bytes_model": bytes_model,
            "avg_launch_ms": round(avg_kernel_s * 1e3, 4), "rays_per_launch": rays_per_launch, **extra}
    pmc = load_json("pmc_%s.json" % run_key(args))
    if pmc and pmc.get("rays_per_launch") and pmc.get("lib_sha256") != lib_sha:
        # counters of another build: they say nothing about the kernel timed here
        roof["counters"] = ("stale: profiles/pmc_%s.json was measured on libsvo_rt.so %s, this run loads %s; traffic, L2 hit "
                            "rate and instruction counts omitted" % (run_key(args), (pmc.get("lib_sha256") or "(unrecorded)")[:12],
                                                                     lib_sha[:12]))
        roof["counters_build"] = pmc.get("lib_sha256")
        pmc = None
    if pmc and pmc.get("rays_per_launch"):
        c = pmc["counters_per_dispatch"]
        scale = rays_per_launch / pmc["rays_per_launch"]  # per-ray figures of the N=1 pass, this launch's rays
        traffic = pmc["hbm_bytes_per_launch"] * scale
        hbm = traffic / avg_kernel_s / 1e9
        valu = c["SQ_INSTS_VALU"] * scale
        valu_frac = valu * VALU_CYCLES / (N_SIMD * CLOCK_GHZ * 1e9 * avg_kernel_s)
        roof.update({
            "traffic": round(traffic), "hbm_gbs_measured": round(hbm, 1), "hbm_frac_measured": round(hbm / HBM_PEAK_GBS, 4),
            "l2_hit_rate": round(pmc["l2_hit_rate"], 4) if pmc.get("l2_hit_rate") is not None else None,
            "valu_insts_per_wave": round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1),
            "salu_insts_per_wave": round(c["SQ_INSTS_SALU"] / c["SQ_WAVES"], 1) if "SQ_INSTS_SALU" in c else None,
            "valu_issue_frac": round(valu_frac, 4),
            "counters": "profiles/pmc_%s.json (rocprofv3 --pmc passes, tools/pmc.sh%s), measured on this build" % (
                run_key(args), "; scaled per ray to this launch" if world > 1 or scale != 1 else ""),
            "counters_build": pmc["lib_sha256"],
            "valu_issue_rule": "SQ_INSTS_VALU x %d cycles / (%d SIMDs x %.1f GHz x launch time)" % (VALU_CYCLES, N_SIMD, CLOCK_GHZ),
        })
        if all(k in c for k in ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")):
            wc = c["SQ_WAVE_CYCLES"]
            roof["limiter"] = ("dependent instruction chains: of the wave-cycles %.0f %% issue, %.0f %% wait to issue, %.0f %% wait on "
                               "memory (SQ counters of the same pass); VALU issue %.2f of peak; measured HBM traffic %.1f %% of peak "
                               "(the nodes the bytes model counts are served from L2 / MALL)"
                               % (100.0 * c["SQ_ACTIVE_INST_ANY"] / wc, 100.0 * c["SQ_WAIT_INST_ANY"] / wc, 100.0 * c["SQ_WAIT_ANY"] / wc,
                                  valu_frac, 100.0 * hbm / HBM_PEAK_GBS))
        else:
            roof["limiter"] = ("instruction stream: VALU issue %.2f of peak, measured HBM traffic %.1f %% of peak (the nodes the model "
                               "counts are served from L2 / MALL)" % (valu_frac, 100.0 * hbm / HBM_PEAK_GBS))
    return roof


# ------------------------------------------------------------------------------- watchdog --
WATCHDOG_RC = 124  # a rank's exit status when its watchdog fires (the status `timeout` gives)


class Watchdog:
    """N > 1: a per-rank guard against a step that never finishes (a receive whose message never comes — a stuck RCCL
    group — leaves every rank waiting, and no rank would ever exit, so launch_ranks' / torchrun's failure handling
    would never fire).  The main thread names its phase as it goes (`phase`: the step and cast / exchange / sync);
    `arm(seconds, what)` sets a deadline.  When one passes, the rank writes which step and phase it is stuck in, the
    state of its last steps' GPU events (cast done / exchange pending, queried with a bounded wait), and every
    thread's Python traceback (faulthandler) to stderr, and leaves with WATCHDOG_RC through os._exit — no re-exec;
    the launcher then ends the other ranks."""

    def __init__(self, rank, world):
        import threading

        self.rank, self.world = rank, world
        self.phase = "start"
        self.deadline = None
        self.what = ""
        self.bound = 0.0
        self.diag = None  # () -> str: the GPU events of the last steps (bench main)
        self.t = threading.Thread(target=self._run, name="bench-watchdog", daemon=True)
        self.t.start()

    def arm(self, seconds, what):
        self.bound = float(seconds)
        self.what = what
        self.deadline = time.monotonic() + self.bound

    def disarm(self):
        self.deadline = None

    def _run(self):
        while True:
            time.sleep(0.1)
            dl = self.deadline
            if dl is not None and time.monotonic() > dl:
                self._fire()

    def _fire(self):
        import faulthandler
        import threading

        err = sys.stderr
        err.write("bench.py: rank %d of %d: WATCHDOG: %s did not finish within %.1f s; stuck in phase: %s\n"
                  % (self.rank, self.world, self.what, self.bound, self.phase))
        err.flush()
        faulthandler.dump_traceback(file=err, all_threads=True)
        err.flush()
        if self.diag is not None:  # (a GPU query could block behind a runtime lock the stuck call holds: bounded)
            out = []
            th = threading.Thread(target=lambda: out.append(self.diag()), daemon=True)
            th.start()
            th.join(3.0)
            err.write("bench.py: rank %d: GPU events of the last steps: %s\n" % (self.rank, out[0] if out else "(query did not return)"))
        err.flush()
        os._exit(WATCHDOG_RC)


def watchdog_bound(warm_s, warm_steps, steps):
    """The timed region's bound from the warm-up's wall time per step (which includes the first launches' and the
    communicator's set-up, so it overestimates a step): SVO_WATCHDOG_FACTOR (default 20) times the steps' expected time,
    at least SVO_WATCHDOG_MIN_S (default 60 s)"""
    per = warm_s / max(1, warm_steps)
    return max(float(os.environ.get("SVO_WATCHDOG_MIN_S", "60")), float(os.environ.get("SVO_WATCHDOG_FACTOR", "20")) * per * (steps + 2))


# ------------------------------------------------------------------------------ rank launcher --
def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, grace_s=30.0, script=None):
    """`python bench.py --gpus N` without a launcher: start N fresh child processes of this script, one
    per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free port), and wait
    for them.  This process touches no GPU (nothing here imports torch), and nothing is exec'd: the
    children are new processes.  Rank 0 prints the JSON line on the inherited stdout.  When a child
    fails, the others get `grace_s` to finish before they are terminated (by PID); the exit status is
    the first failing child's (a signal: 128 + its number)."""
    import signal
    import subprocess

    env0 = dict(os.environ)
    env0.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                GROUP_RANK="0", ROLE_RANK="0", TORCHELASTIC_RUN_ID="bench_%d" % os.getpid())
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), ROLE_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env))
    rc, t_fail = 0, None
    while True:
        codes = [p.poll() for p in procs]
        for c in codes:
            if c is not None and c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                t_fail = time.monotonic()
        if all(c is not None for c in codes):
            break
        if t_fail is not None and time.monotonic() - t_fail > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
            t_kill = time.monotonic()
            while any(p.poll() is None for p in procs) and time.monotonic() - t_kill < 10.0:
                time.sleep(0.1)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            break
        time.sleep(0.05)
    if rc:
        print("bench.py: a rank failed (exit status %d); see its stderr" % rc, file=sys.stderr)
    return rc


# ------------------------------------------------------------------------------------- main --
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="c3: depth-12 / 1080p (the metric); c5: depth-14 / 4K; c2: the reference world / 1080p / S=300 from the "
                         "C3 pose, c2cam0 from the reference's default camera; c1: the dense 256^3 grid, 256^2 rays")
    ap.add_argument("--inflight", type=int, choices=(1, 2), default=1,
                    help="2: consecutive steps' casts alternate between two streams, so two frames are in flight on every rank "
                         "(the next frame's long far-field waves fill this one's tail; a small shard of a strong-scaled frame "
                         "gains most); the line's launch times are then each launch's own, overlapped")
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per step over all GPUs (strong scaling; default: one per GPU, weak scaling)")
    ap.add_argument("--ao", type=int, default=0, help="config C4: hemisphere AO rays per primary hit (16 or 20)")
    ap.add_argument("--shade", action="store_true",
                    help="SURVEY §8f.1: shaded frames (svo_shade_rays: primary + reflections + 75-step sun shadow ray)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 CPU timing inside cpu_baseline")
    ap.add_argument("--no-gather", action="store_true", help="N>1: cast only, no exchange")
    ap.add_argument("--exchange", default="capi", choices=["capi", "torch"],
                    help="capi: svo_exchange_frames (RCCL inside libsvo_rt); torch: all_to_all_single of wire records")
    ap.add_argument("--force-exchange", action="store_true", help="run the exchange at N=1 too (a one-rank RCCL communicator)")
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--origin", default=None, help="camera position x,y,z (default: the config's; e.g. a non-integral one)")
    ap.add_argument("--iterative", action="store_true", help="A/B: voxel-by-voxel DDA (SVO_CAST_ITERATIVE)")
    ap.add_argument("--stats", action="store_true", help="print traversal counters of one extra frame to stderr")
    ap.add_argument("--cast-flags", type=int, default=0, help="extra SVO_CAST_* bits (experiments)")
    ap.add_argument("--host-build", action="store_true", help="build the tree on the host (default: svo_build_terrain_gpu)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal on one GPU; torch exchange)")
    ap.add_argument("--verify", action="store_true",
                    help="with an exchange at N = 1 (--force-exchange): check the displayed frames against a one-GPU cast "
                         "of them (at N > 1 this is the default)")
    ap.add_argument("--no-verify", action="store_true",
                    help="N > 1: skip the check of the displayed frames after the timed region (gather_verified null)")
    ap.add_argument("--pipelined-steps", type=int, default=None,
                    help="N = 1: after the timed region, time this many more steps with consecutive launches on two "
                         "alternating streams (a launch's tail overlaps the next one's head), reported as `pipelined` "
                         "(default: --steps; 0: off)")
    ap.add_argument("--launch-events", action="store_true",
                    help="an event pair around every cast launch (default at N=1: one pair around the timed region, whose "
                         "average per launch includes the gaps between launches; per-launch pairs cost ~7 us per step)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher around us: start the ranks ourselves, before anything touches a GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        ap.error("WORLD_SIZE=%s (from the launcher) differs from --gpus %d" % (env_world, args.gpus))

    import torch
    import torch.distributed as dist

    import raytracing_test_amd as rt
    from raytracing_test_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if world > 1 and args.dist_backend == "nccl" and world > ndev:
        ap.error("%d ranks over RCCL need %d GPUs (%d visible); --dist-backend gloo rehearses N ranks on fewer" % (world, world, ndev))
    dev = local % max(1, ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)
    wd = Watchdog(rank, world) if world > 1 else None
    if wd:  # (set-up: the tree build, buffers, the communicator)
        wd.arm(float(os.environ.get("SVO_WATCHDOG_SETUP_S", "600")), "set-up (tree build, exchange communicator)")
    cfg = dict(CONFIGS[args.config])
    if args.cols is not None:
        cfg["cols"] = args.cols
    if args.origin is not None:
        cfg["origin"] = tuple(float(v) for v in args.origin.split(","))
    W, H, STEPS = cfg["W"], cfg["H"], cfg["steps"]
    if args.shade and args.ao:
        ap.error("--shade and --ao are separate workloads")

    # ---- the tree, resident in HBM before timing
    t0 = time.time()
    builder = "gpu"
    if args.config == "c1":  # the reference world's [0,256)^3, voxel by voxel (product getBlock / putBlock)
        ref = rt.World.reference()
        g = np.stack(np.meshgrid(np.arange(256), np.arange(256), np.arange(256), indexing="ij"), -1).reshape(-1, 3).astype(np.int32)
        bf, bc, _ = ref.get_blocks(g)
        stored = bc != np.uint64(0xFFFFFFFFFFFFFFFF)
        w4 = rt.World(4)
        w4.put_blocks(g[stored], bf[stored] & ~np.uint32(1), bc[stored])
        tree = w4.build()
        builder = "host (putBlock)"
        build_s = time.time() - t0
        tree.upload(dev)
    elif args.config == "c2d8":  # a clean depth-8 root + genWorld, putBlock by putBlock
        w8 = rt.World(4)
        w8.gen_world(200, 200)
        tree = w8.build()
        builder = "host (putBlock)"
        build_s = time.time() - t0
        tree.upload(dev)
    elif args.config.startswith("c2"):  # initTetraHexaTree + genWorld, putBlock by putBlock
        tree = rt.World.reference().build()
        builder = "host (putBlock)"
        build_s = time.time() - t0
        tree.upload(dev)
    elif args.host_build:
        tree = rt.Tree.terrain(cfg["levels"], cfg["cols"], cfg["cols"], nthreads=16)
        builder = "host"
        build_s = time.time() - t0
        tree.upload(dev)
    else:  # noise + build in HBM (identical arrays, tests/test_gpu_build.py); already uploaded
        tree = rt.Tree.terrain_gpu(cfg["levels"], cfg["cols"], cfg["cols"], dev)
        build_s = time.time() - t0
    scene = None
    if args.shade:  # the shading scene: every block, water included (it refracts, low_res.frag:214-229)
        if args.config in ("c1", "c2", "c2cam0", "c2d8"):
            scene = {"c1": lambda: w4, "c2d8": lambda: w8}.get(args.config, rt.World.reference)().build(rt.VIEW_ALL).upload(dev)
        elif args.host_build:
            scene = rt.Tree.terrain(cfg["levels"], cfg["cols"], cfg["cols"], nthreads=16, view=rt.VIEW_ALL).upload(dev)
        else:
            scene = rt.Tree.terrain_gpu(cfg["levels"], cfg["cols"], cfg["cols"], dev, view=rt.VIEW_ALL)
    info = tree.info()
    ppx, ppy = rt.proj_plane(W, H)
    cam = rt.normalize(cfg["cam"])

    # ---- frames of a step and this rank's shard of them (one launch covers the shard of every frame)
    strong = args.frames is not None
    nframes = args.frames if strong else world
    if not 1 <= nframes <= 16:
        ap.error("1 <= frames per step <= 16 (SVO_MAX_FRAMES)")
    origins = [frame_origin(cfg, f) for f in range(nframes)]
    flags = (rt.CAST_ITERATIVE if args.iterative else 0) | args.cast_flags
    desc = rt.Tree.frame_desc(origins[0], cam, W, H, STEPS, ppx, ppy, tile_row_start=rank, tile_row_step=world, flags=flags,
                              ao_samples=args.ao, frame_origins=origins if nframes > 1 else None)
    rays_per_launch = rt.Tree.count(desc)
    gather = (world > 1 or args.force_exchange) and not args.no_gather
    xmode = None
    # the C-ABI exchange needs RCCL; a gloo rehearsal takes it too when SVO_RCCL_LIB names the test-only stand-in
    # (tests/standin/rccl_standin.cpp: several ranks on one GPU, host-staged), else the torch exchange
    # (the library honours SVO_RCCL_LIB only with SVO_RCCL_STANDIN=1 as well)
    standin = (os.environ.get("SVO_RCCL_LIB") or None) if os.environ.get("SVO_RCCL_STANDIN") == "1" else None
    if gather:
        xmode = "torch" if (args.shade or args.exchange == "torch" or (args.dist_backend != "nccl" and not standin)) else "capi"
    # tensors for the small control collectives: on the GPU over RCCL, on the host over gloo
    gdev = torch.device("cuda", dev)
    cdev = gdev if args.dist_backend == "nccl" else torch.device("cpu")
    pipe_steps = args.steps if args.pipelined_steps is None else args.pipelined_steps
    if gather or world > 1 or args.inflight > 1:
        pipe_steps = 0  # (an N = 1 measurement beside the contract's own)
    # the exchange (or the next launch) of step k overlaps step k+1.  With an exchange, three buffer sets: step k's
    # decode runs beside cast k+1 and gets wave slots only in that cast's tail, so cast k+2 reusing step k's buffers would
    # wait for it (a bubble every step: the 1-rank exchange's k_wire_scatter spans 150 us of the 173-us cast beside it)
    nbuf = 3 if gather else (2 if (pipe_steps or args.inflight > 1) else 1)
    outs = []
    for _ in range(nbuf):
        views = rt.Tree.alloc_hits(rays_per_launch, dev, ao=args.ao > 0)
        if args.shade:
            views["rgba"] = torch.zeros((rays_per_launch, 4), dtype=torch.float32, device=gdev)
        outs.append(views)
    cstreams = [torch.cuda.Stream(device=dev) for _ in range(2 if (pipe_steps or args.inflight > 1) else 1)]
    inflight = args.inflight > 1  # the timed steps alternate between the two cast streams (two frames in flight)
    stream = cstreams[0]
    xstream = torch.cuda.Stream(device=dev) if gather else None
    exch = None
    xnote = None
    n_own = len(range(rank, nframes, world))  # frames this rank displays
    frames_out = None
    if xmode == "capi":
        try:
            if world > 1:
                uid = torch.zeros(rt.NCCL_UNIQUE_ID_BYTES, dtype=torch.uint8, device=cdev)
                if rank == 0:
                    uid.copy_(torch.frombuffer(bytearray(rt.Exchange.unique_id()), dtype=torch.uint8))
                dist.broadcast(uid, 0)
                uid = bytes(uid.cpu().numpy().tobytes())
            else:
                uid = rt.Exchange.unique_id()
            exch = rt.Exchange(world, rank, uid, dev)
            if exch.info() != (rank, world):
                raise RuntimeError("svo_exchange_info reports rank/size %s, expected (%d, %d)" % (exch.info(), rank, world))
        except rt.SvoError as e:  # keep the scaling run alive; say so on the line
            xmode, xnote = "torch", "svo_exchange_create failed (%s); torch.distributed all_to_all used" % e
        if world > 1:
            # every rank takes the same path: a rank whose exchange failed would otherwise wait in all_to_all while the
            # others wait in RCCL send / recv
            ok = torch.tensor([1 if exch is not None else 0], dtype=torch.int32, device=cdev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and exch is not None:
                torch.cuda.synchronize()
                exch.close()
                exch = None
                xmode, xnote = "torch", "svo_exchange_create failed on another rank; torch.distributed all_to_all used"
        if exch is not None and n_own:
            frames_out = rt.Tree.alloc_hits(n_own * W * H, dev, ao=args.ao > 0)
    # the C-ABI exchange casts straight into wire records (svo_cast_wire: 8 B per ray from integral camera
    # positions, else 12 B) and decodes them on the display rank (svo_exchange_wire): no hit records, no pack
    wires = None
    if exch is not None:
        wb = tree.wire_bytes(desc)
        wires = [torch.empty((rays_per_launch, wb), dtype=torch.uint8, device=gdev) for _ in range(nbuf)]

    # torch exchange (shading image, gloo rehearsal, or --exchange torch): frame f -> rank f % world
    counts = [shard.shard_count(W, H, r, world) for r in range(world)]
    n_mine = counts[rank]
    offs = np.concatenate([[0], np.cumsum(counts)]).tolist()
    tx = None
    if xmode == "torch":
        tx = TorchExchange(args, rt, tree, dist, torch, gdev, W, H, STEPS, ppx, ppy, cam, origins, rank, world, counts, offs, n_mine,
                           outs, nbuf)

    xdone = [None] * nbuf
    # N > 1: the last steps' cast / exchange events (the watchdog's report; per-step events, not per buffer set)
    recent = collections.deque(maxlen=6)

    def events_state():
        def st(e):
            return "-" if e is None else ("done" if e.query() else "PENDING")
        return "; ".join("step %d: cast %s, exchange %s" % (k, st(c), st(x)) for k, c, x in list(recent)) or "(no step issued)"

    if wd:
        wd.diag = events_state

    def one_step(k, ev=None, pipe=False):
        b = k % nbuf
        stream = cstreams[k % 2] if pipe else cstreams[0]
        if wd:
            wd.phase = "step %d: cast (svo_cast%s)" % (k, "_wire" if wires is not None else "_rays")
        with torch.cuda.stream(stream):
            if xdone[b] is not None:
                stream.wait_event(xdone[b])  # the exchange that read this buffer set has passed
            if ev is not None:
                ev[0].record(stream)
            if args.shade:
                # the image is the product: no hit records, so rays that provably leave the scene upwards stop early
                tree.shade(desc, outs[b]["rgba"], out=None, stream=stream, scene=scene)
            elif wires is not None:
                tree.cast_wire(desc, wires[b], outs[b].get("ao"), stream)
            else:
                tree.cast(desc, outs[b], stream)
            if ev is not None:
                ev[1].record(stream)
        ce = None
        if wd or xmode == "capi":
            ce = torch.cuda.Event()
            ce.record(stream)
        if not gather:
            if wd:
                recent.append((k, ce, None))
            return
        if wd:
            wd.phase = "step %d: exchange (%s)" % (k, "svo_exchange_wire: RCCL send / recv group, decode" if xmode == "capi"
                                                   else "torch.distributed all_to_all")
        if xmode == "capi":
            xstream.wait_event(ce)
            exch.wire(tree, desc, wires[b], frames_out, ao=outs[b].get("ao"), stream=xstream)
            e = torch.cuda.Event()
            e.record(xstream)
            xdone[b] = e
        else:
            xdone[b] = tx.step(k, b, stream)
        if wd:
            recent.append((k, ce, xdone[b]))
            wd.phase = "step %d: issued" % k

    def drain():
        if tx is not None:
            tx.drain(stream)

    step_no = 0
    if wd:
        wd.arm(float(os.environ.get("SVO_WATCHDOG_WARMUP_S", "300")), "the warm-up steps")
    tw = time.perf_counter()
    n_warm = max(args.warmup, 2) if inflight else args.warmup
    for _ in range(n_warm):
        one_step(step_no, pipe=inflight)
        step_no += 1
    if wd:
        wd.phase = "warm-up: draining (synchronize: waiting for the GPU)"
    drain()
    torch.cuda.synchronize()
    if world > 1:
        wd.phase = "warm-up: barrier"
        dist.barrier()
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw
    if wd:
        wd.arm(watchdog_bound(warm_s, n_warm, args.steps), "the timed region (%d steps)" % args.steps)
    evs = [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(args.steps)]
    reg = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    # one event pair around the timed region on the cast stream gives the average launch (gaps and the waits for the
    # exchange included); timing events around every launch (--launch-events) would serialise the cast and exchange
    # streams (1-rank exchange: 0.197 ms per step with them, ~0.175 without — tools/xchg_host.py)
    # (two frames in flight: the pair spans both cast streams — the second waits for the opening event, the first for the
    # second's last launch before the closing one)
    region_events = not args.launch_events
    t0 = time.perf_counter()
    if region_events:
        reg[0].record(stream)
        if inflight:
            cstreams[1].wait_event(reg[0])
    for k in range(args.steps):
        one_step(step_no, None if region_events else evs[k], pipe=inflight)
        step_no += 1
    if region_events:
        if inflight:
            j = torch.cuda.Event()
            j.record(cstreams[1])
            stream.wait_event(j)
        reg[1].record(stream)
    if wd:
        wd.phase = "timed region: draining (synchronize: waiting for the GPU)"
    drain()
    torch.cuda.synchronize()
    if world > 1:
        wd.phase = "timed region: barrier"
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if wd:
        wd.arm(float(os.environ.get("SVO_WATCHDOG_POST_S", "300")), "the per-rank timing and the frame check after the timed region")
        wd.phase = "after the timed region"
    kern_ms = [reg[0].elapsed_time(reg[1]) / args.steps] if region_events else [e[0].elapsed_time(e[1]) for e in evs]
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_rays = W * H * nframes * args.steps  # every rank's share of every frame, all steps
    value = total_rays / elapsed
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    pipelined = None
    if pipe_steps:
        # the same steps with consecutive launches on two alternating streams: frames are independent, so a
        # renderer keeps two in flight and the next launch's long waves fill this one's tail
        for _ in range(max(2, args.warmup)):  # (the second stream's first launches set up its queue)
            one_step(step_no, None, pipe=True)
            step_no += 1
        torch.cuda.synchronize()
        pe = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tp = time.perf_counter()
        pe[0].record(cstreams[0])
        cstreams[1].wait_event(pe[0])
        for k in range(pipe_steps):
            one_step(step_no, None, pipe=True)
            step_no += 1
        pe[1].record(cstreams[1])
        cstreams[0].wait_event(pe[1])
        pe[2].record(cstreams[0])
        torch.cuda.synchronize()
        tp = time.perf_counter() - tp
        pipelined = {"value": round(W * H * nframes * pipe_steps / tp, 1), "ms_per_step": round(tp / pipe_steps * 1e3, 4),
                     "event_ms_per_step": round(pe[0].elapsed_time(pe[2]) / pipe_steps, 4), "steps": pipe_steps,
                     "how": "consecutive launches alternate between two streams (two frames in flight); each launch "
                            "itself runs longer, sharing the GPU: the per-launch roofline above is the one-at-a-time figure"}

    per_rank = None
    if world > 1:
        per_rank = rank_timing(args, rt, torch, dist, tree, desc, outs, wires, exch, tx, xmode, gather, frames_out, cstreams[0],
                               xstream, xdone, nbuf, step_no, nframes, W, H, dev, cdev, wd, drain, scene)
        step_no += min(args.steps, 5)

    verified = None
    # N > 1: one step's displayed frames against a one-GPU cast of them, after the timed region, by default
    if (args.verify or (world > 1 and not args.no_verify)) and gather and not args.shade:
        torch.cuda.synchronize()
        ok = True
        for k, f in enumerate(range(rank, nframes, world)):
            one = rt.decode_hits(tree.cast_frame(origins[f], cam, W, H, STEPS, ppx, ppy, flags=flags, ao_samples=args.ao))
            if xmode == "capi":
                got = rt.decode_hits({key: v[k * W * H:(k + 1) * W * H] for key, v in frames_out.items()})
                ok &= all(np.array_equal(got[key], one[key]) for key in got)
            else:
                ok &= tx.verify(f, one)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        verified = bool(flag.item())

    if args.stats and rank == 0:
        print_stats(rt, tree, desc, outs[0], stream, torch)

    # the job's size as the communicators report it: the C-ABI exchange's RCCL communicator
    # (svo_exchange_info), else the torch.distributed group
    n_gpus = exch.info()[1] if exch is not None else (dist.get_world_size() if world > 1 else 1)
    if wd:
        wd.disarm()
    if exch is not None:  # the RCCL communicator of the exchange goes before the process group's
        torch.cuda.synchronize()
        exch.close()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    roof = roofline(args, cfg, rays_per_launch, avg_kernel_s, world, rt.lib_sha256())
    roof["timed_build"] = rt.lib_sha256()
    cpu = None
    if world == 1 and nframes == 1 and not args.no_cpu_baseline:
        gpu = None
        if args.shade:
            gpu = {"rgba": outs[0]["rgba"].cpu().numpy()}
        else:
            gpu = rt.decode_hits(outs[0])
        cpu = cpu_baseline(args, cfg, ppx, ppy, gpu)
    work = ("C4 (C3 + %d hemisphere AO rays per hit, 5 steps each): " % args.ao if args.ao else "") + \
           ("shaded (low_res.frag colour model, water refracts (SVO_VIEW_ALL scene), 75-step shadow rays): " if args.shade else "")
    metric = cfg["metric"]
    if args.ao:
        metric = "primary rays/sec at 1080p with %d-sample hemisphere AO per hit, depth-12 SVO (config 4); achieved HBM GB/s vs roofline" % args.ao
    if args.shade:
        metric = "shaded primary rays/sec (reflections, refraction by water, sun shadow ray)"
    line = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: the reference world (initTetraHexaTree + genWorld on 200x200 columns), built in-process"
                 if args.config in ("c1", "c2", "c2cam0") else
                 "synthetic: a clean depth-8 root + genWorld on 200x200 columns, built in-process" if args.config == "c2d8" else
                 "synthetic: genWorld OpenSimplex terrain (seeds 42/64/100) on %dx%d columns, built in-process" % (cfg["cols"], cfg["cols"])),
        "config": {"workload": work + cfg["label"] + " primary rays per frame, camera (%g,%g,%g)->normalize(%g,%g,%g), S=%d, "
                                                     "castRayFromCam semantics" % (cfg["origin"] + cfg["cam"] + (STEPS,)),
                   "ao_samples": args.ao, "shade": args.shade, "frames_per_step": nframes, "rays_per_step": W * H * nframes,
                   "parallelism": "tile-row shard x%d" % world, "launches_per_step": 1, "frames_in_flight": args.inflight, "gather": gather,
                   "dispatch_order": ("top tile rows first" if not args.shade or (flags & rt.CAST_NO_SCHEDULE) or tree.blocks(desc) <= rt.SCHED_MIN_BLOCKS else
                                      "longest first by a recent frame's block durations (sorted after every 4th frame), in groups of "
                                      "4 blocks (frame schedule, gated on camera motion; the warmup's first two frames: top tile rows "
                                      "first)"),
                   "exchange": None if not gather else (
                       ("svo_cast_wire + svo_exchange_wire (C ABI, RCCL send/recv group): %d-B wire records written by the cast "
                        "kernel" % tree.wire_bytes(desc) + (" + AO counts" if args.ao else "") +
                        ", frame f to rank f % N (own shards decoded in place), decoded on arrival on a second stream "
                        "overlapping the next cast" + (" — transport: the TEST-ONLY host-staged RCCL stand-in (SVO_RCCL_LIB=%s), "
                                                        "not RCCL" % os.path.basename(standin) if standin else ""))
                       if xmode == "capi" else
                       ("torch.distributed all_to_all_single: " + ("rgba image" if args.shade else "12-B wire hit records") +
                        ", frame f to rank f % N" + ("; " + xnote if xnote else ""))),
                   "tree_nodes": info.n_nodes, "tree_bytes": info.n_nodes * 16 + info.n_mat_bytes, "tree_build_s": round(build_s, 3),
                   "tree_builder": builder, **({"scene_nodes": scene.info().n_nodes} if scene is not None else {})},
        "roofline": roof,
        "cpu_baseline": cpu,
        # what carried the exchange: "rccl" (librccl.so.1 inside the C ABI), "standin" (the TEST-ONLY host-staged stand-in:
        # never multi-GPU evidence), "torch" (torch.distributed) or null (no exchange)
        "transport": None if not gather else ("standin" if standin else "rccl") if xmode == "capi" else "torch",
        "build": build_block(rt),
        **({"gather_verified": verified} if (verified is not None or world > 1) else {}),
        **({"gather_verify_note": "the shaded image's exchange is not checked (gather_verified null)" if args.shade else
            "--no-verify" if args.no_verify else "no exchange (--no-gather)"} if verified is None and world > 1 else {}),
        **({"pipelined": pipelined} if pipelined is not None else {}),
        **({"per_rank": per_rank} if per_rank is not None else {}),
        "launch_timing": "one HIP event pair around the timed region on the launch stream (average per launch, gaps "
                         "included" + ("; two frames in flight: the pair spans both cast streams" if inflight else "") + ")"
                         if region_events else "a HIP event pair around every launch on its stream (--launch-events)",
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def build_block(rt):
    """The timed library's provenance: its file hash, the sources_sha256 stamped into it at build time (svo_build_id),
    that stamp recomputed from the source files present here, and whether they agree (a stale library would not)"""
    from raytracing_test_amd import build as B

    stamp = rt.build_id()
    try:
        here = B.sources_sha256()
    except OSError:
        here = None
    return {"libsvo_rt_sha256": rt.lib_sha256(), "library": os.path.relpath(rt.LIB_PATH, ROOT),
            "sources_sha256": stamp, "sources_sha256_recomputed": here,
            "sources_match": (stamp is not None and stamp == here) if "SVO_LIB" not in os.environ else None}


def rank_timing(args, rt, torch, dist, tree, desc, outs, wires, exch, tx, xmode, gather, frames_out, stream, xstream, xdone, nbuf,
                step_no, nframes, W, H, dev, cdev, wd, drain, scene):
    """N > 1, after the timed region: every rank's own cost, so a slow rank in a scaling run can be named.  A few more
    steps with an event pair around each cast (cast stream) and each C-ABI exchange (its stream: the RCCL send / recv
    group plus the decode of the shards received), then the decode alone: svo_wire_scatter of this rank's own shard,
    the display rank's cost per source shard.  Medians in ms; all ranks' figures are gathered to rank 0."""
    nd = min(args.steps, 5)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    cast_ms, xch_ms, dec_ms = [], [], []
    pairs = []
    for i in range(nd):
        k = step_no + i
        b = k % nbuf
        if wd:
            wd.phase = "per-rank timing, step %d: cast" % k
        c0, c1 = ev(), ev()
        with torch.cuda.stream(stream):
            if xdone[b] is not None:
                stream.wait_event(xdone[b])
            c0.record(stream)
            if wires is not None:
                tree.cast_wire(desc, wires[b], outs[b].get("ao"), stream)
            elif args.shade:
                tree.shade(desc, outs[b]["rgba"], out=None, stream=stream, scene=scene)
            else:
                tree.cast(desc, outs[b], stream)
            c1.record(stream)
        x0 = x1 = None
        if gather:
            if wd:
                wd.phase = "per-rank timing, step %d: exchange" % k
            if xmode == "capi":
                x0, x1 = ev(), ev()
                xstream.wait_event(c1)
                x0.record(xstream)
                exch.wire(tree, desc, wires[b], frames_out, ao=outs[b].get("ao"), stream=xstream)
                x1.record(xstream)
                xdone[b] = x1
            else:
                xdone[b] = tx.step(k, b, stream)
        pairs.append((c0, c1, x0, x1))
    if wd:
        wd.phase = "per-rank timing: synchronize"
    drain()
    torch.cuda.synchronize()
    for c0, c1, x0, x1 in pairs:
        cast_ms.append(c0.elapsed_time(c1))
        if x0 is not None:
            xch_ms.append(x0.elapsed_time(x1))
    if wires is not None:
        if wd:
            wd.phase = "per-rank timing: decode"
        scratch = rt.Tree.alloc_hits(nframes * W * H, dev, ao=args.ao > 0)
        for _ in range(3):
            d0, d1 = ev(), ev()
            d0.record(stream)
            tree.wire_scatter(desc, wires[0], scratch, ao=outs[0].get("ao"), stream=stream)
            d1.record(stream)
            torch.cuda.synchronize()
            dec_ms.append(d0.elapsed_time(d1))
        del scratch
    med = lambda v: float(np.median(v)) if v else float("nan")
    mine = torch.tensor([med(cast_ms), med(xch_ms), med(dec_ms)], dtype=torch.float64, device=cdev)
    allr = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    if wd:
        wd.phase = "per-rank timing: all_gather"
    dist.all_gather(allr, mine)
    rows = []
    for r, t in enumerate(allr):
        c, x, d = (float(v) for v in t.cpu().numpy())
        rows.append({"rank": r, "cast_ms": round(c, 4), "exchange_ms": None if x != x else round(x, 4),
                     "decode_shard_ms": None if d != d else round(d, 4)})
    return {"ranks": rows, "steps": nd,
            "how": "after the timed region: median of %d steps with an event pair around each cast (cast stream) and each "
                   "C-ABI exchange (its stream: RCCL send / recv group + decode of the shards received); decode_shard_ms = "
                   "svo_wire_scatter of this rank's own shard alone (the display rank's decode cost per source shard)" % nd}


class TorchExchange:
    """The exchange through torch.distributed (the shaded image, gloo rehearsals, --exchange torch):
    frame f's tile-row shards to rank f % N by one all_to_all_single per buffer, wire records packed
    by svo_hits_pack and unpacked by svo_hits_unpack on arrival."""

    def __init__(self, args, rt, tree, dist, torch, gdev, W, H, STEPS, ppx, ppy, cam, origins, rank, world, counts, offs, n_mine, outs,
                 nbuf):
        self.a, self.rt, self.tree, self.dist, self.torch = args, rt, tree, dist, torch
        self.W, self.H, self.world, self.rank = W, H, world, rank
        self.counts, self.offs, self.n_mine = counts, offs, n_mine
        self.nframes = len(origins)
        self.nbuf = nbuf
        self.wire = not args.shade
        self.outs = outs
        # frames sent per destination rank: frame f -> rank f % world; receive my frames from every rank
        self.mine = list(range(rank, self.nframes, world))
        self.desc = rt.Tree.frame_desc(origins[0], cam, W, H, STEPS, ppx, ppy, tile_row_start=rank, tile_row_step=world,
                                       frame_origins=origins if self.nframes > 1 else None)
        self.src_descs = {f: [rt.Tree.frame_desc(origins[f], cam, W, H, STEPS, ppx, ppy, tile_row_start=r, tile_row_step=world)
                              for r in range(world)] for f in self.mine}
        # one record per row, svo_wire_bytes(desc) wide (8 B compact from integral / half-integral camera positions,
        # else 12 B): the all-to-all splits count records, so the rows must be the packed stride.  Every frame's own
        # shard descs must agree with the launch's format (the configs shift their frames by whole voxels)
        self.wb = tree.wire_bytes(self.desc)
        if any(tree.wire_bytes(d) != self.wb for ds in self.src_descs.values() for d in ds):
            raise RuntimeError("frames of one launch with different wire formats (integral and fractional camera positions)")
        self.sends, self.recvs = [], []
        for b in range(nbuf):
            snd, rcv = [], []
            if self.wire:
                snd.append(torch.zeros((n_mine * self.nframes, self.wb), dtype=torch.uint8, device=gdev))
                rcv.append(torch.zeros((max(1, len(self.mine)) * W * H, self.wb), dtype=torch.uint8, device=gdev))
            if args.ao:
                snd.append(outs[b]["ao"])
                rcv.append(torch.zeros(max(1, len(self.mine)) * W * H, dtype=torch.uint8, device=gdev))
            if args.shade:
                snd.append(outs[b]["rgba"])
                rcv.append(torch.zeros((max(1, len(self.mine)) * W * H, 4), dtype=torch.float32, device=gdev))
            self.sends.append(snd)
            self.recvs.append(rcv)
        self.host = args.dist_backend != "nccl"
        self.recv_host = [[torch.empty_like(x, device="cpu") for x in r] for r in self.recvs] if self.host else None
        self.frames = rt.Tree.alloc_hits(max(1, len(self.mine)) * W * H, gdev.index) if self.wire else None
        self.pending = {}

    def _splits(self, elems_per_record):
        """all_to_all_single splits: my records of frame f go to rank f % N (frames in order); I receive
        my frames' shards from every rank, frame by frame"""
        send = [0] * self.world
        for f in range(self.nframes):
            send[f % self.world] += self.n_mine * elems_per_record
        recv = [sum(self.counts[r] for _ in self.mine) * elems_per_record for r in range(self.world)]
        return send, recv

    def _order_send(self, x):
        # records of frame f at f * n_mine: regroup by destination rank (frames f, f + N, ... per rank)
        idx = [f for r in range(self.world) for f in range(r, self.nframes, self.world)]
        if idx == list(range(self.nframes)):
            return x
        n = self.n_mine
        return self.torch.cat([x[f * n:(f + 1) * n] for f in idx])

    def step(self, k, b, stream):
        torch, dist = self.torch, self.dist
        with torch.cuda.stream(stream):
            if self.wire:
                self.tree.pack_hits(self.desc, self.outs[b], self.sends[b][0], stream)
            works, keep = [], []
            for i, (snd, rcv) in enumerate(zip(self.sends[b], self.recvs[b])):
                s_split, r_split = self._splits(1)
                src = self._order_send(snd)
                src = src if not self.host else src.cpu()
                dst = rcv if not self.host else self.recv_host[b][i]
                dst = dst[:sum(r_split)]
                works.append(dist.all_to_all_single(dst, src, output_split_sizes=r_split, input_split_sizes=s_split, async_op=True))
                keep.append(src)
            self.pending[k] = (works, keep, b)
            if (k - 1) in self.pending:
                self._unpack(k - 1, stream)
        return None

    def _unpack(self, k, stream):
        works, _, b = self.pending.pop(k)
        for w in works:
            w.wait()
        if self.host:
            for i, h in enumerate(self.recv_host[b]):
                self.recvs[b][i].copy_(h)
        if not self.wire:
            return
        # received layout: from rank r, its shards of my frames in order
        base = 0
        for r in range(self.world):
            for j, f in enumerate(self.mine):
                lo = j * self.W * self.H + self.offs[r]
                part = {key: v[lo:lo + self.counts[r]] for key, v in self.frames.items()}
                self.tree.unpack_hits(self.src_descs[f][r], self.recvs[b][0][base:base + self.counts[r]], part, stream)
                base += self.counts[r]

    def drain(self, stream):
        with self.torch.cuda.stream(stream):
            for k in sorted(self.pending):
                self._unpack(k, stream)

    def verify(self, f, one):
        """frame f (displayed here) reassembled from the shards == a one-GPU cast of it"""
        from raytracing_test_amd import shard

        j = self.mine.index(f)
        got = self.rt.decode_hits({key: v[j * self.W * self.H:(j + 1) * self.W * self.H] for key, v in self.frames.items()})
        ok = True
        for r in range(self.world):
            rows = shard.shard_pixel_rows(self.H, r, self.world)
            idx = (rows[:, None] * self.W + np.arange(self.W)[None, :]).reshape(-1)
            lo = self.offs[r]
            ok &= all(np.array_equal(got[key][lo:lo + self.counts[r]], one[key][idx]) for key in ("pos", "steps", "hit", "axis", "material", "t"))
        return ok


def print_stats(rt, tree, d0, out, stream, torch):
    nblk = rt.Tree.blocks(d0)
    for mode in (rt.CAST_STATS, rt.CAST_TIMELINE):
        st = torch.zeros(rt.STATS_HEADER + 2 * nblk + rt.Tree.count(d0), dtype=torch.int64, device=out["t"].device)
        d0.flags |= mode
        d0.stats = st.data_ptr()
        tree.cast(d0, out, stream)
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
        if os.environ.get("SVO_STAMPS"):  # per-block start / end stamps (dispatch order) for offline analysis
            np.save(os.environ["SVO_STAMPS"], stamps)
        stamps = stamps[stamps[:, 1] > 0].astype(np.float64) / 100.0  # launched blocks; us (100 MHz)
        if len(stamps) == 0:  # (the AO instances keep no timeline)
            continue
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


if __name__ == "__main__":
    main()
