#!/bin/bash
# parity suite (cast, large tree, shading, edits), then A/B of library variants on several configs:
#   tools/gpu_ab_multi.sh <tag> <lib|default>...   (CONFIGS="...": bench-arg sets separated by ';')
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_shade.py tests/test_gpu_edits.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
IFS=';' read -ra CFGS <<< "${CONFIGS:- ;--ao 16;--config c5;--config c3f}"
i=0
for c in "${CFGS[@]}"; do
  i=$((i+1)); echo "== $c"
  BENCH_ARGS="$c" REPS=${REPS:-4} bash tools/ab_lib.sh ${TAG}_$i "$@" || exit 1
done
