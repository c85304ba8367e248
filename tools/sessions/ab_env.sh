#!/bin/bash
# A/B timing of environment settings in one GPU session: tools/ab_env.sh <tag> "<VAR=val ...>"...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
for E in "$@"; do
  n=$(echo "$E" | tr ' =' '__')
  env $E timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/ab_$n.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/ab_$n.json'));print('env=%s rep=$rep ms=%.4f Grays/s=%.3f'%('$E',d['roofline']['avg_launch_ms'],d['value']/1e9))"
done
done
