"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) for the cast kernel k_cast.

HBM bytes per launch = FETCH_SIZE * 2 (gfx950: FETCH_SIZE reports half the bytes of 128-B reads,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB per dispatch.  The factor-2 correction is
calibrated on wide streaming reads; the cast kernel issues 16-B node gathers, so the raw FETCH_SIZE is
kept beside it."""
import csv
import glob
import json
import os
import sys


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def per_dispatch(d, kernel="k_cast"):
    vals = {}
    for r in rows(d):
        if kernel not in r.get("Kernel_Name", ""):
            continue
        key = (r.get("Dispatch_Id"), r["Counter_Name"])
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    agg = {}
    for (disp, name), v in vals.items():
        agg.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def bench_line(out):
    """the bench JSON line of a pass (its rays per launch)"""
    for f in sorted(glob.glob(os.path.join(out, "pmc_*.log"))):
        for line in open(f):
            if line.startswith("{"):
                try:
                    return json.loads(line)
                except ValueError:
                    pass
    return None


def main(out, bench_args=""):
    res = {"kernel": "k_cast", "source": out, "bench_args": bench_args}
    counters = {}
    for d in sorted(glob.glob(os.path.join(out, "pmc_*")) + glob.glob(os.path.join(out, "sq_*"))):
        if os.path.isdir(d):
            c, n = per_dispatch(d)
            counters.update(c)
    res["counters_per_dispatch"] = counters
    fetch = counters.get("FETCH_SIZE")
    write = counters.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        res["fetch_kib_raw"] = fetch
        res["write_kib"] = write
        res["hbm_bytes_per_launch"] = (2.0 * fetch + write) * 1024.0
        res["hbm_bytes_per_launch_uncorrected"] = (fetch + write) * 1024.0
    h, m = counters.get("TCC_HIT_sum"), counters.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m > 0:
        res["l2_hit_rate"] = h / (h + m)
    b = bench_line(out)
    # the build the passes ran (bench.py's line): bench.py reads these counters only for the same libsvo_rt.so
    res["lib_sha256"] = (b or {}).get("build", {}).get("libsvo_rt_sha256")
    if b and b.get("roofline"):
        res["rays_per_launch"] = b["roofline"]["rays_per_launch"]
        res["bench_avg_launch_ms"] = b["roofline"]["avg_launch_ms"]
    elif counters.get("SQ_WAVES"):
        res["rays_per_launch"] = counters["SQ_WAVES"] * 64  # one 64-lane wave per 16x4 footprint
    if counters.get("SQ_WAVES") and counters.get("SQ_INSTS_VALU"):
        res["valu_per_wave"] = counters["SQ_INSTS_VALU"] / counters["SQ_WAVES"]
        if counters.get("SQ_INSTS_SALU"):
            res["salu_per_wave"] = counters["SQ_INSTS_SALU"] / counters["SQ_WAVES"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
