#!/bin/bash
# A/B timing of (environment, cast flags) pairs in one GPU session, interleaved repetitions:
#   tools/ab_cfg.sh <tag> "<VAR=val ...>:<flags>"...      e.g. ":0" "SVO_REFILL=16:64"   (REPS=3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 ${REPS:-3}); do
for C in "$@"; do
  E=${C%%:*}; F=${C##*:}
  n=$(echo "${E}_f$F" | tr ' =/.' '____')
  env $E timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --cast-flags $F ${BENCH_ARGS:-} > gpurun_out/$TAG/ab_${n}_$rep.json 2>/dev/null || exit 1
done
done
python3 - "$TAG" "$@" <<'PY'
import json, sys, glob, statistics
tag = sys.argv[1]
for C in sys.argv[2:]:
    E, F = C.split(':')
    n = ('%s_f%s' % (E, F))
    for ch in ' =/.': n = n.replace(ch, '_')
    ms = [json.load(open(f))['roofline']['avg_launch_ms'] for f in sorted(glob.glob('gpurun_out/%s/ab_%s_*.json' % (tag, n)))]
    print('cfg=%-28s ms min %.4f median %.4f  (%s)' % (C, min(ms), statistics.median(ms), ' '.join('%.4f' % m for m in ms)))
PY
