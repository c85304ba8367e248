#!/bin/bash
# r04 session K: dispatch order of the single-pass shading kernel (lake rows sit ~60 % down the frame): top first
# (default), bottom first, 8x8 tiles; and the split shading bottom first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_k; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
for v in "1 0" "1 4" "1 256" "2 4"; do
  set -- $v
  timeout -k 10 120 python bench.py --shade --no-cpu-baseline --steps 30 --shade-passes $1 --cast-flags $2 > $OUT/s$1_f$2_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$OUT/s$1_f$2_$rep.json')); print('passes $1 flags $2', d['ms_per_step'])"
done
done
