#!/bin/bash
# r03 session H: C3 per-block stamps + per-pixel work (launch-tail analysis), C4 AO-20 plan loads (bytes model)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_h; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_h] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $OUT/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
run stats_c3 300 env SVO_STAMPS=$OUT/stamps_c3.npy SVO_RAY_WORK=$OUT/work_c3.npy python -u bench.py --stats --steps 5 --warmup 2 --no-cpu-baseline
run stats_c4_ao20 300 python -u bench.py --stats --ao 20 --steps 5 --warmup 2 --no-cpu-baseline
run stats_c4_ao16 300 python -u bench.py --stats --ao 16 --steps 5 --warmup 2 --no-cpu-baseline
