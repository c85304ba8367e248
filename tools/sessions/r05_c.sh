#!/bin/bash
# r05_c: per-block stamps + per-ray work of one C3 frame (STATS / TIMELINE instances), and the top-rows probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_c; mkdir -p $OUT
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/bench.json 2> $OUT/stats.txt || exit 1
timeout -k 10 300 python tools/tail_probe.py > $OUT/tail_probe.txt 2>&1 || exit 1
cat $OUT/stats.txt $OUT/tail_probe.txt | tail -30
