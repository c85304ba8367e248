#!/bin/bash
# r03 session I: the launch's critical path — top tile rows cast alone vs the full frame; issue priority for
# the top tile rows (A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_i; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_i] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $OUT/$name.log | cut -c1-800; [ $rc -eq 0 ] || exit $rc; }
run probe 300 python -u tools/tail_probe.py
run ab_prio 900 env REPS=4 bash tools/ab_lib.sh r03_i_prio default variants/libsvo_prio4.so variants/libsvo_prio12.so variants/libsvo_prio34.so
