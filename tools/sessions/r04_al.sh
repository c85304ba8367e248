#!/bin/bash
# r04 session AL: three buffer sets with an exchange: the 1-rank RCCL exchange lines (C3, C5 --frames 1, C4) against two
# (git stash of bench.py is not available on the box: --nbuf-exchange is not an option, so HEAD's bench.py is compared via
# its copy bench_nbuf2.py), the gather tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_al; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for b in bench bench_nbuf2; do
  timeout -k 10 120 python $b.py --force-exchange --verify --no-cpu-baseline --steps 30 > $OUT/c3_${b}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python $b.py --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline --steps 20 > $OUT/c5_${b}_$rep.json 2>/dev/null || exit 1
done
done
python3 - <<'PY'
import json, glob, statistics
for c in ('c3', 'c5'):
    for b in ('bench', 'bench_nbuf2'):
        ds = [json.loads([l for l in open(f) if l.startswith('{')][-1]) for f in sorted(glob.glob('gpurun_out/r04_al/%s_%s_*.json' % (c, b)))]
        ms = [d['ms_per_step'] for d in ds]
        print(c, b, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms), 'verified', all(d.get('gather_verified') for d in ds))
PY
