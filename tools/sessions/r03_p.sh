#!/bin/bash
# r03 session P: segmented rays for the top tile rows — parity with every row segmented (SVO_SPLIT_ROWS=100000), then
# the A/B of split-row counts and lanes per ray on C3 / C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_p; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_p] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -8 $OUT/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run pytest_all_split 900 env SVO_SPLIT_ROWS=100000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_bridge.py tests/test_gpu_edits.py -m gpu -x -q --timeout 300 --timeout-method thread
V="default variants/libsvo_split4.so variants/libsvo_split8.so variants/libsvo_split16.so variants/libsvo_split8k2.so variants/libsvo_split16k2.so variants/libsvo_split32k2.so"
run ab_c3 900 env REPS=3 bash tools/ab_lib.sh r03_p_c3 $V
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_p_c5 $V
