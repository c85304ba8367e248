#!/bin/bash
# r03 session G: gpu tests with ballot-gated ceiling exits in the shading instances only; A/B against the
# all-gated build (variants/libsvo_gate.so) on C3, C5, shaded C3; then the round's evidence session
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_g; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_g] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
L="variants/libsvo_gate.so default"
run ab_c3 900 env REPS=6 bash tools/ab_lib.sh r03_g_c3 $L
run ab_c5 900 env REPS=3 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_g_c5 $L
run ab_shade 900 env REPS=3 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_g_sh $L
bash tools/evidence.sh r03ev
