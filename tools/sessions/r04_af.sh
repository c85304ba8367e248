#!/bin/bash
# r04 session AF: the 1-rank exchange's step cost with the cast streams at high priority against normal (C3, C5 --frames 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_af; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3 4; do
for p in 0 1; do
  timeout -k 10 120 python bench.py --force-exchange --no-cpu-baseline --steps 30 --cast-priority $p > $OUT/c3_p${p}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py --config c5 --frames 1 --force-exchange --no-cpu-baseline --steps 20 --cast-priority $p > $OUT/c5_p${p}_$rep.json 2>/dev/null || exit 1
done
done
python3 - <<'PY'
import json, glob, statistics
for c in ('c3', 'c5'):
    for p in (0, 1):
        ms = [json.loads([l for l in open(f) if l.startswith('{')][-1])['ms_per_step'] for f in sorted(glob.glob('gpurun_out/r04_af/%s_p%d_*.json' % (c, p)))]
        print(c, 'priority', p, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms))
PY
