#!/bin/bash
# rocprofv3 kernel traces (one-at-a-time launches: --pipelined-steps 0) and the bench lines that
# depend on committed counters.  usage: tools/evidence_prof.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-evp}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1; shift; echo "[evidence] $(date +%T) $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for c in "c3:" "c3f:--config c3f" "c4:--ao 16" "c5:--config c5" "shade:--shade"; do
  n=${c%%:*}; a=${c#*:}
  step prof_$n timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- python3 bench.py $a --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_$n.json 2> $OUT/prof_$n.err
  grep -h "k_cast" $OUT/prof_$n/run_kernel_stats.csv | cut -c1-160
done
step c3f timeout -k 10 300 python bench.py --config c3f > $OUT/bench_c3f.json 2> $OUT/bench_c3f.err
