#!/bin/bash
# r04 session AG: the parts of the shaded frame at the round's build (tools/shade_parts.py), and its counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ag; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_parts.py > $OUT/parts.log 2>&1 || { tail $OUT/parts.log; exit 1; }
grep -v amdgpu.ids $OUT/parts.log
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
