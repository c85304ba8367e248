#!/bin/bash
# rocprofv3 PMC passes for the cast kernel (one counter group per pass, no trace domains — see
# MI355X_MICROARCH.md §HBM / rocprofv3 PMC slots).  Writes gpurun_out/<tag>/pmc_*/ and the summary
# profiles-ready JSON gpurun_out/<tag>/pmc_traffic.json.  usage: tools/pmc.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $*"  # extra args: another config
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$i" -o run -- $BENCH > "$OUT/pmc_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/pmc_traffic.json"
cat "$OUT/pmc_traffic.json"
