#!/bin/bash
# r03 session L (re-entry): gpu tests on the rebuilt tree; the launch's critical path — C3 with the top K tile rows
# dropped (SVO_DROP_TOP, diagnostics) and the per-block stamps of the STATS build (tile-row durations)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_l; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_l] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run stamps 300 env SVO_STAMPS=$OUT/stamps_c3.npy python -u bench.py --stats --steps 5 --warmup 2 --no-cpu-baseline
run ab_drop 900 env REPS=3 bash tools/ab_lib.sh r03_l_drop default variants/libsvo_drop4.so variants/libsvo_drop8.so variants/libsvo_drop16.so
