#!/bin/bash
# A/B of library variants on one bench configuration: tools/gpu_ab_cfg.sh <tag> "<bench args>" <lib|default>...
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; ARGS=$2; shift 2
BENCH_ARGS="$ARGS" REPS=${REPS:-4} bash tools/ab_lib.sh $TAG "$@"
