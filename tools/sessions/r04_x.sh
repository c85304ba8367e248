#!/bin/bash
# r04 session X: two-phase shading (the frame octant's primary code first, bent rays traced again) on the LDS-bounce
# 5-wave instance, against HEAD; its shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_x; mkdir -p $OUT; export TMPDIR=/tmp
SVO_LIB=$PWD/variants/libsvo_twophase.so timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_x/ab variants/libsvo_base.so variants/libsvo_twophase.so || exit 1
