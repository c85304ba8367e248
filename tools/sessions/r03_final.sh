#!/bin/bash
# r03 final evidence (run as r03_final at d127496, r03_final2 at the ceiling-pair build, r03_final3 at the packed-pair build, r03_final4 with the box gates): the full gpu suite, then tools/evidence.sh (bench lines of every config with CPU baselines,
# the 1-rank RCCL exchange, gloo rehearsals, rocprofv3 kernel traces)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_final4; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r03_final] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/evidence.sh r03_final4
