#!/bin/bash
# r04 session Z: the gather tests (incl. two frames in flight), C5 strong-mode lines at N = 1 with one and two frames in
# flight, the shaded line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_z; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --frames 1 --inflight $f --no-cpu-baseline > $OUT/c5_strong_if$f.json 2> $OUT/c5_if$f.err || { tail $OUT/c5_if$f.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c5_strong_if$f.json')); print('c5 frames1 inflight $f', d['ms_per_step'], round(d['value']/1e9,2))"
done
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python -c "import json; d=json.load(open('$OUT/shade.json')); print('shade', d['ms_per_step'], d['roofline']['frac'])"
