#!/bin/bash
# r05_i: clock probe — far-field waves alone vs inside the whole frame: duration, shader cycles, clock
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_i; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_clock.so timeout -k 10 300 python tools/clock_probe.py > $OUT/clock_probe.txt 2> $OUT/clock_probe.err; rc=$?
cat $OUT/clock_probe.txt; tail -3 $OUT/clock_probe.err; exit $rc
