#!/bin/bash
# r03 session M: the launch tail — C3 launch time and rays cut with a per-ray iteration cap (SVO_ITER_CAP variants)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_m; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_m] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc; }
run default 300 python -u tools/cap_probe.py
for m in 16 24 32 48; do run cap$m 300 env SVO_LIB=$PWD/variants/libsvo_cap$m.so python -u tools/cap_probe.py; done
