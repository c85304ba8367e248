#!/bin/bash
# rocprofv3 PMC passes for the cast kernel k_cast (one counter group per pass, kernel counters only, no
# trace domains — MI355X_MICROARCH.md §HBM / rocprofv3 PMC slots).  Writes gpurun_out/<tag>/pmc_*/ and
# the summary gpurun_out/<tag>/pmc_summary.json (copy to profiles/pmc_<config>.json, which bench.py reads).
# usage: tools/pmc.sh <tag> [bench args, e.g. --ao 16 / --config c5 / --shade]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$i" -o run -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --pipelined-steps 0 "$@" > "$OUT/pmc_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" "$*" > "$OUT/pmc_summary.json"
cat "$OUT/pmc_summary.json"
