#!/bin/bash
# r04 session E: shaded frame, ceiling levels 64/256 (working tree) against 16/64 (variants/libsvo_shade1664.so) now that
# rays above the tree's top cross one global box; the parts of the shaded frame (tools/shade_parts.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_e; mkdir -p $OUT; export TMPDIR=/tmp
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_e/ab variants/libsvo_shade1664.so default || exit 1
timeout -k 10 300 python tools/shade_parts.py > $OUT/parts.log 2>&1; rc=$?; cat $OUT/parts.log; exit $rc
