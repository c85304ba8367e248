#!/bin/bash
# A/B of library variants on the default (integral) camera, then the fractional camera (current lib)
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-abf}; shift
mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
REPS=${REPS:-4} bash tools/ab_lib.sh $TAG "$@" || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --origin 4.37,90.61,4.23 > gpurun_out/$TAG/frac.json 2> gpurun_out/$TAG/frac.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/frac.json')); print('fractional camera ms', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
