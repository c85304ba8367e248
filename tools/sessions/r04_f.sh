#!/bin/bash
# r04 session F: the shading pass walking every ceiling level (max-mipmap, P.ceilq): shading / edits / small-tree tests,
# then A/B against HEAD (libsvo_base) and the global box with 16/64 pairs (libsvo_shade1664); shading counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_f; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_f] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py tests/test_gpu_edits.py tests/test_gpu_small_trees.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_f] $(date +%T) A/B"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_f/ab variants/libsvo_base.so variants/libsvo_shade1664.so default || exit 1
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
