#!/bin/bash
# r03 session O: issue priority raised by a wave's traversal iterations (SVO_PRIO_IT variants), C3 and C5 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_o; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_o] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $OUT/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
V="default variants/libsvo_prio8.so variants/libsvo_prio12.so variants/libsvo_prio16.so variants/libsvo_prio24.so"
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_o_c3 $V
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_o_c5 $V
