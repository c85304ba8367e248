#!/bin/bash
# r04 session AV: block timelines after the shading schedule (primary: default order) (tools/shade_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_av; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_timeline.py gpurun_out/r04_av/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
cat $OUT/timeline.json
