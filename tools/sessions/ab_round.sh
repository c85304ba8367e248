#!/bin/bash
# GPU parity suite, then interleaved A/B timing of library variants: tools/ab_round.sh <tag> <lib.so|default>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
REPS=${REPS:-3} timeout -k 10 900 bash tools/ab_lib.sh $TAG "$@"
