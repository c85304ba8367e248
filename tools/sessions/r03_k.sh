#!/bin/bash
# r03 session K: 16/64-column ceilings for primary casts, 64/256 for shading (runtime levels): gpu tests, A/B
# against the session-G library (variants/libsvo_r03i.so = commit 65b0c5a) on C3 / C5 / shaded / C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_k; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_k] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
L="variants/libsvo_r03i.so default"
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_k_c3 $L
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_k_c5 $L
run ab_shade 900 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_k_sh $L
run ab_c4 900 env REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r03_k_c4 $L
run ab_c3f 900 env REPS=2 BENCH_ARGS="--config c3f" bash tools/ab_lib.sh r03_k_c3f $L
