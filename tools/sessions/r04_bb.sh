#!/bin/bash
# r04 session BB: primary casts under the grouped, camera-gated frame schedule (a variant that attaches it to primary
# and AO launches too) against the shipped default order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04_bb; export TMPDIR=/tmp
REPS=3 bash tools/ab_lib.sh r04_bb/c3 default variants/libsvo_prim_sched.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r04_bb/c5 default variants/libsvo_prim_sched.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r04_bb/c4 default variants/libsvo_prim_sched.so || exit 1
