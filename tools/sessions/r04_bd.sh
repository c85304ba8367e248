#!/bin/bash
# r04 session BD: the shading schedule by groups of 8 blocks (variant) against groups of 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04_bd; export TMPDIR=/tmp
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r04_bd/shade default variants/libsvo_sched_g8.so || exit 1
