#!/bin/bash
# r04 session U: the shading instance without segment-exact crossings (SEG false: integral cameras' rays stay linear, also
# after refraction) against HEAD; its shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_u; mkdir -p $OUT; export TMPDIR=/tmp
SVO_LIB=$PWD/variants/libsvo_shadenoseg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_u/ab variants/libsvo_base.so variants/libsvo_shadenoseg.so || exit 1
