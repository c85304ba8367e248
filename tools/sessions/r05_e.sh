#!/bin/bash
# r05_e: critical-path probe — far-field waves with fewer rays per wave (tools/lane_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_e; mkdir -p $OUT
timeout -k 10 600 python tools/lane_probe.py > $OUT/lane_probe.txt 2> $OUT/lane_probe.err; rc=$?
tail -1 $OUT/lane_probe.txt; tail -3 $OUT/lane_probe.err; exit $rc
