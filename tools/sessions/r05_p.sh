#!/bin/bash
# r05_p: after the march — the top tile rows alone (critical path) and the per-block timeline / per-ray work of C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_p; mkdir -p $OUT
timeout -k 10 200 python tools/tail_probe.py --reps 10 > $OUT/tail.txt 2>/dev/null || exit 1
tail -1 $OUT/tail.txt
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/stats.json 2> $OUT/stats.txt || exit 1
grep "stats per ray\|timeline" $OUT/stats.txt
