#!/bin/bash
# r03 session A: gpu tests (new full-frame / depth-8 / half-integral cases), budget-guard A/B against
# the round-start library, exchange parts at C5, AO plan loads and budget counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_a; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_a] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run ab 900 env REPS=4 bash tools/ab_lib.sh r03_a_ab variants/libsvo_base.so variants/libsvo_nopass.so default
run xchg_c5 300 python tools/xchg_parts.py --config c5
run xchg_c3 300 python tools/xchg_parts.py --config c3 --shards 2
run stats_c3 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --pipelined-steps 0 --stats
run stats_c4 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --pipelined-steps 0 --stats --ao 16
