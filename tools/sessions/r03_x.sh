#!/bin/bash
# r03 session X: with the forward-box gate, also gate the ceiling box exits by a ballot of the lanes above their ceiling
# (SVO_CEIL_GATE=1, variants/libsvo_cgate1.so): its gpu tests, A/B on C3 / C5 / shaded / C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_x; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_x] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
L="default variants/libsvo_cgate1.so"
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_x_c3 $L
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_x_c5 $L
run ab_shade 900 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_x_sh $L
run ab_c4 900 env REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r03_x_c4 $L
run pytest_cgate1 600 env SVO_LIB=$PWD/variants/libsvo_cgate1.so python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
