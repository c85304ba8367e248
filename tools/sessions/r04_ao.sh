#!/bin/bash
# r04 session AO: the exchange's decode in one-wave blocks (it runs beside the next cast): forced 1-rank exchange lines
# against HEAD (libsvo_base); the wire / gather tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ao; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "wire or exchange" tests/test_gpu_bench_gather.py tests/test_gpu_bridge.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--force-exchange --verify" timeout -k 10 600 bash tools/ab_lib.sh r04_ao/c3 variants/libsvo_base.so default || exit 1
REPS=3 BENCH_ARGS="--config c5 --frames 1 --force-exchange --verify" timeout -k 10 600 bash tools/ab_lib.sh r04_ao/c5 variants/libsvo_base.so default || exit 1
