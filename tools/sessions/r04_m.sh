#!/bin/bash
# r04 session M: the shading instance's bounce state (and origin / direction) in LDS instead of spilled registers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_m; mkdir -p $OUT; export TMPDIR=/tmp
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_m/ab variants/libsvo_base.so variants/libsvo_ldsboth.so variants/libsvo_ldsbn.so || exit 1
