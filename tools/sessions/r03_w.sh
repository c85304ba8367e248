#!/bin/bash
# r03 session W: forward boxes skipped when every crossing lane of the wave takes a ceiling box (wave-uniform ballot; a
# whole-air iteration): gpu tests, A/B against the ungated build (variants/libsvo_gate0.so) on C3 / C5 / shaded / C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_w; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_w] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
L="variants/libsvo_gate0.so default"
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_w_c3 $L
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_w_c5 $L
run ab_shade 900 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_w_sh $L
run ab_c4 900 env REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r03_w_c4 $L
