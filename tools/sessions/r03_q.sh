#!/bin/bash
# r03 session Q: segmented rays with early stop (a segment ends once an earlier segment of its ray hit): parity with
# every row segmented, A/B of split rows / lanes per ray / floor against the unsplit build (nostop)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_q; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_q] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -9 $OUT/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run pytest_all_split 900 env SVO_SPLIT_ROWS=100000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_bridge.py tests/test_gpu_edits.py -m gpu -x -q --timeout 300 --timeout-method thread
V="variants/libsvo_nostop.so default variants/libsvo_s8.so variants/libsvo_s8k2.so variants/libsvo_s8f24.so variants/libsvo_s16f24.so"
run ab_c3 900 env REPS=3 bash tools/ab_lib.sh r03_q_c3 $V
