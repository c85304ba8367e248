#!/bin/bash
# r03 session E: column-ceiling variants (levels checked, per-lane ceiling cache) on C3, C5 and shaded C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_e2; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_e] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
L="variants/libsvo_base.so default variants/libsvo_l1.so variants/libsvo_c2.so variants/libsvo_c1.so"
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_e_c3 $L
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_e_c5 $L
run ab_shade 900 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_e_sh $L
