#!/bin/bash
# The full GPU suite + smoke + default bench line (tools/gpu_full.sh), then an interleaved A/B of
# library variants:  tools/gpu_full_ab.sh <tag> <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
timeout -k 10 1000 bash tools/gpu_full.sh $TAG || exit $?
REPS=${REPS:-4} timeout -k 10 600 bash tools/ab_lib.sh ${TAG}_ab "$@"
