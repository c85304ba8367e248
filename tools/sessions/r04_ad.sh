#!/bin/bash
# r04 session AD: the 8-wave AO instance (table from the kernel arguments, no start barrier): the AO / parity tests, then
# C4, C3 and shaded A/B against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ad; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--ao 16" timeout -k 10 600 bash tools/ab_lib.sh r04_ad/c4 variants/libsvo_base.so default || exit 1
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_ad/c3 variants/libsvo_base.so default || exit 1
REPS=3 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_ad/shade variants/libsvo_base.so default || exit 1
