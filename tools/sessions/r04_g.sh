#!/bin/bash
# r04 session G: shading counters with refraction passes, the long tail of bent rays
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
