#!/bin/bash
# SQ stall breakdown of the cast kernel (separate --pmc passes, kernel counters only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sq}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
BENCH="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $*"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SMEM" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/sq_$i" -o run -- $BENCH > "$OUT/sq_$i.log" 2>&1 || { echo "pass $i failed"; tail -3 $OUT/sq_$i.log; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" | python3 -c "
import json,sys; d=json.load(sys.stdin)['counters_per_dispatch']
for k in sorted(d): print('%-32s %16.1f' % (k, d[k]))
"
