#!/bin/bash
# r04 session P: the refractive pass continuing into sibling bricks: shading tests, A/B against HEAD, counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_p; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_p] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_p/ab variants/libsvo_base.so default || exit 1
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
