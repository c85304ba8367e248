#!/bin/bash
# r04 session Y: shadow rays crossing the scene's column-ceiling boxes (CEIL 1), against HEAD; shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_y; mkdir -p $OUT; export TMPDIR=/tmp
SVO_LIB=$PWD/variants/libsvo_shadowceil.so timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_y/ab variants/libsvo_base.so variants/libsvo_shadowceil.so || exit 1
