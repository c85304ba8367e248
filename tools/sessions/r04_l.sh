#!/bin/bash
# r04 session L: the shading instance of the frame's octant casting with the primary's code first (bent rays traced again):
# shading tests, A/B against HEAD (libsvo_base: one reflecting instance for every ray)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_l; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_l] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py tests/test_gpu_bridge.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_l/ab variants/libsvo_base.so default || exit 1
