#!/bin/bash
# r03 session N: per-block stamps and per-ray work (lookups, iterations, brick steps, node loads) of one C3 frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_n; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_n] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
run stats 300 env SVO_STAMPS=$OUT/stamps_c3.npy SVO_RAY_WORK=$OUT/work_c3.npy python -u bench.py --stats --steps 5 --warmup 2 --no-cpu-baseline
