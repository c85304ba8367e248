#!/bin/bash
# r04 final evidence: the GPU suite, then tools/evidence.sh (every config's bench line with its CPU baseline, the 1-rank
# RCCL exchange, gloo rehearsals, rocprofv3 kernel traces), then the C3 PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${R04_FINAL_TAG:-r04_final}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_final] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/evidence.sh ${R04_FINAL_TAG:-r04_final}/ev || exit $?
bash tools/pmc.sh ${R04_FINAL_TAG:-r04_final}/pmc_c3 > $OUT/pmc_c3.log 2>&1 || { tail $OUT/pmc_c3.log; exit 1; }
tail -3 $OUT/pmc_c3.log
