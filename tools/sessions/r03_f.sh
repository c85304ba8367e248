#!/bin/bash
# r03 session F: gpu tests with the cached, ballot-gated column ceilings; A/B against the round-start library and
# the ungated cached build (c2) on C3, C5, shaded C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_f; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_f] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
L="variants/libsvo_base.so variants/libsvo_c2.so default"
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_f_c3 $L
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_f_c5 $L
run ab_shade 900 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_f_sh $L
run c2d8 300 python -u bench.py --config c2d8 --steps 50 --warmup 10
