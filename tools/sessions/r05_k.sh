#!/bin/bash
# r05_k: where the shaded frame's time goes now: plain cast, shaded with / without shadow rays, without water
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_k; mkdir -p $OUT
timeout -k 10 300 python tools/shade_parts.py > $OUT/shade_parts.txt 2> $OUT/shade_parts.err; rc=$?
cat $OUT/shade_parts.txt; exit $rc
