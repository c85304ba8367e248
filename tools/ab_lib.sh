#!/bin/bash
# A/B timing of library variants (SVO_LIB) in one GPU session: tools/ab_lib.sh <tag> <lib.so|default>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/$L; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/ab_$n.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/ab_$n.json'));print('lib=%s rep=$rep ms=%.4f Grays/s=%.3f'%('$n',d['roofline']['avg_launch_ms'],d['value']/1e9))"
done
done
