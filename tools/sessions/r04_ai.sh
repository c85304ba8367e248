#!/bin/bash
# r04 session AI: wavefront footprint per config — 16x4 (default), 8x8 (flag 256), 32x2 (flag 512) at C3, C5, C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ai; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
for cfg in "c3" "c5" "c3 --ao 16"; do
for fl in 0 256 512; do
  tag=$(echo "$cfg" | tr -d ' -')
  timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 30 --cast-flags $fl > $OUT/${tag}_f${fl}_$rep.json 2>/dev/null || exit 1
done
done
done
python3 - <<'PY'
import json, glob, statistics
for tag in ('c3', 'c5', 'c3ao16'):
    for fl in (0, 256, 512):
        ms = [json.load(open(f))['roofline']['avg_launch_ms'] for f in sorted(glob.glob('gpurun_out/r04_ai/%s_f%d_*.json' % (tag, fl)))]
        print(tag, 'flags', fl, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms))
PY
