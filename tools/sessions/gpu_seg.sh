#!/bin/bash
# segment-exact crossings: parity tests, fractional-camera stats, A/B on the default (integral) camera
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-seg}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shade.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for o in 4.37,90.61,4.23 4.0,90.0,4.0; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --steps 10 --stats --origin $o > $OUT/b_$o.json 2> $OUT/err_$o.log || exit 1
  grep -E "stats" $OUT/err_$o.log | cut -c1-330; cut -c1-200 $OUT/b_$o.json
done
REPS=4 bash tools/ab_lib.sh ${1:-seg}_ab variants/libsvo_head.so default
