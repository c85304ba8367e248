#!/bin/bash
# r03 session B: brick pass-through variants A/B (gated by a wave ballot: full box test, y-rows test)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_b; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_b] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run ab 900 env REPS=4 bash tools/ab_lib.sh r03_b_ab variants/libsvo_nopass.so variants/libsvo_passF.so variants/libsvo_passY.so
run stats_F 300 env SVO_LIB=$PWD/variants/libsvo_passF.so python bench.py --no-cpu-baseline --steps 3 --warmup 1 --pipelined-steps 0 --stats
run stats_Y 300 env SVO_LIB=$PWD/variants/libsvo_passY.so python bench.py --no-cpu-baseline --steps 3 --warmup 1 --pipelined-steps 0 --stats
run c4 300 python bench.py --no-cpu-baseline --steps 10 --ao 16 --pipelined-steps 0
