#!/bin/bash
# A/B timing of svo_cast_desc.flags variants in one GPU session, interleaved repetitions:
#   tools/ab_flags.sh <tag> <flags>...        (REPS=4 by default; BENCH_ARGS extra bench.py args)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 ${REPS:-4}); do
for F in "$@"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --cast-flags $F ${BENCH_ARGS:-} > gpurun_out/$TAG/abf_${F}_$rep.json 2>/dev/null || exit 1
done
done
python3 - "$TAG" "$@" <<'PY'
import json, sys, glob, statistics
tag = sys.argv[1]
for F in sys.argv[2:]:
    ds = [json.load(open(f)) for f in sorted(glob.glob('gpurun_out/%s/abf_%s_*.json' % (tag, F)))]
    ms = [d['roofline']['avg_launch_ms'] if d.get('roofline') else d['ms_per_step'] for d in ds]
    print('flags=%-6s ms min %.4f median %.4f  (%s)' % (F, min(ms), statistics.median(ms), ' '.join('%.4f' % m for m in ms)))
PY
