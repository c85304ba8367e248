#!/bin/bash
# r04 session AN: bench.py timing the region with one event pair on the cast stream(s) also with an exchange / two
# frames in flight (per-launch timing events serialised the streams): forced 1-rank exchange lines against HEAD's
# bench.py (bench_old.py), the gather tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_an; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for b in bench bench_old; do
  timeout -k 10 120 python $b.py --force-exchange --verify --no-cpu-baseline --steps 30 > $OUT/c3_${b}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python $b.py --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline --steps 20 > $OUT/c5_${b}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python $b.py --config c5 --frames 1 --inflight 2 --no-cpu-baseline --steps 20 > $OUT/c5if_${b}_$rep.json 2>/dev/null || exit 1
done
done
python3 - <<'PY'
import json, glob, statistics
for c in ('c3', 'c5', 'c5if'):
    for b in ('bench', 'bench_old'):
        ds = [json.loads([l for l in open(f) if l.startswith('{')][-1]) for f in sorted(glob.glob('gpurun_out/r04_an/%s_%s_[0-9].json' % (c, b)))]
        ms = [d['ms_per_step'] for d in ds]
        print(c, b, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms), 'verified', [d.get('gather_verified') for d in ds],
              'avg_launch', ds[0]['roofline']['avg_launch_ms'])
PY
