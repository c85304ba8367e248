#!/bin/bash
# r03 session D: column ceilings — gpu tests, A/B against the round-start library and against the
# SVO_CAST_NO_CEILINGS flag (C3, C5, shaded C3), traversal counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_d; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_d] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run ab 900 env REPS=4 bash tools/ab_lib.sh r03_d_ab variants/libsvo_base.so default
run abf_c3 600 env REPS=3 bash tools/ab_flags.sh r03_d_abf 0 32768
run abf_c5 600 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_flags.sh r03_d_abf5 0 32768
run abf_shade 600 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_flags.sh r03_d_abfs 0 32768
run stats_c3 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --pipelined-steps 0 --stats
