#!/bin/bash
# r04 session BC: host time of edit + update + sync (tools/edit_sync_timing.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_bc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/edit_sync_timing.py > $OUT/edit_sync.json 2> $OUT/edit_sync.err || { tail $OUT/edit_sync.err; exit 1; }
cat $OUT/edit_sync.json
