#!/bin/bash
# A/B timing of library variants (SVO_LIB) in one GPU session, interleaved repetitions:
#   tools/ab_lib.sh <tag> <lib.so|default>...        (REPS=4 by default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 ${REPS:-4}); do
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/$L; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS:-} > gpurun_out/$TAG/ab_${n}_$rep.json 2>/dev/null || exit 1
done
done
python3 - "$TAG" "$@" <<'PY'
import json, sys, glob, statistics, os
tag = sys.argv[1]
for L in sys.argv[2:]:
    n = os.path.basename(L)[:-3] if L.endswith('.so') else L
    # (the last JSON line: an RCCL exchange prints its banner to stdout first)
    ds = [json.loads([l for l in open(f) if l.startswith('{')][-1]) for f in sorted(glob.glob('gpurun_out/%s/ab_%s_*.json' % (tag, n)))]
    ms = [d['roofline']['avg_launch_ms'] if d.get('roofline') else d['ms_per_step'] for d in ds]  # (shaded: no roofline)
    print('lib=%-22s ms min %.4f median %.4f  (%s)' % (n, min(ms), statistics.median(ms), ' '.join('%.4f' % m for m in ms)))
PY
