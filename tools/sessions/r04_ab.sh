#!/bin/bash
# r04 session AB: far-field tile rows (the first K dispatched) crossing 64 / 256-column ceiling boxes instead of 16 / 64
# (experiment library libsvo_far, SVO_FAR_ROWS = K), C3 and C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ab; mkdir -p $OUT; export TMPDIR=/tmp
export SVO_LIB=$PWD/variants/libsvo_far.so
for cfg in c3 c5; do
for rep in 1 2 3; do
for K in 0 8 16 32 64; do
  SVO_FAR_ROWS=$K timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 30 > $OUT/${cfg}_k${K}_$rep.json 2>/dev/null || exit 1
done
done
python3 - $cfg <<'PY'
import json, glob, statistics, sys
cfg = sys.argv[1]
for K in (0, 8, 16, 32, 64):
    ms = [json.load(open(f))['roofline']['avg_launch_ms'] for f in sorted(glob.glob('gpurun_out/r04_ab/%s_k%d_*.json' % (cfg, K)))]
    print(cfg, 'K=%d' % K, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms))
PY
done
