#!/bin/bash
# r04 session AS: the shaded frame's per-block timeline (tools/shade_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_as; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_timeline.py gpurun_out/r04_as/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
cat $OUT/timeline.json
