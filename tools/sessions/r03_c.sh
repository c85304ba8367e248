#!/bin/bash
# r03 session C: gpu tests (wire formats, scatter of N > 1 shards, fused exchange), progress-guard and XCD
# footprint-grouping A/B against the round-start library, shading at 7 waves, exchange parts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_c; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_c] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run ab 900 env REPS=4 bash tools/ab_lib.sh r03_c_ab variants/libsvo_base.so variants/libsvo_guard2.so variants/libsvo_xcd4.so variants/libsvo_xcd16.so variants/libsvo_xcd60.so
run ab_shade 900 env REPS=3 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_c_abs variants/libsvo_guard2.so variants/libsvo_shade7.so
run xchg_c5 300 python tools/xchg_parts.py --config c5
run xchg_c3 300 python tools/xchg_parts.py --config c3 --shards 8
run c5x 300 python bench.py --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline --steps 10
run c3x 300 python bench.py --force-exchange --verify --no-cpu-baseline --steps 10
