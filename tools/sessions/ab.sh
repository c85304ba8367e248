#!/bin/bash
# A/B timing of cast flag variants in one GPU session: tools/ab.sh <tag> <flags...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
for f in "$@"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --cast-flags $f > gpurun_out/$TAG/ab_$f.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/ab_$f.json'));print('flags=%s rep=$rep ms=%.4f Grays/s=%.3f'%('$f',d['roofline']['avg_launch_ms'],d['value']/1e9))"
done
done
