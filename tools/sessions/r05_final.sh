#!/bin/bash
# r05 final evidence: the GPU suite, smoke, then tools/evidence.sh (every config's bench line with its CPU baseline, the
# 1-rank RCCL exchange, gloo rehearsals, the C-ABI exchange at N = 2 / 3 over the test-only stand-in, rocprofv3 kernel
# traces) on the library whose PMC passes are in profiles/pmc_*.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${R05_FINAL_TAG:-r05_final}; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
echo "[r05_final] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/evidence.sh ${R05_FINAL_TAG:-r05_final}/ev || exit $?
