#!/bin/bash
# One GPU call: VALU counts + interleaved A/B timing of library variants, plus C3 traversal stats.
#   tools/gpu_ab_now.sh <tag> <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
if [ -n "${STATS:-}" ]; then
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --stats > gpurun_out/$TAG/stats.json 2> gpurun_out/$TAG/stats.err || exit 1
  grep "per ray" gpurun_out/$TAG/stats.err | cut -c1-1500
fi
timeout -k 10 600 bash tools/pmc_valu.sh $TAG "$@" || exit 1
REPS=${REPS:-4} timeout -k 10 900 bash tools/ab_lib.sh $TAG "$@"
