#!/bin/bash
# r04 session A: the launcher-free 2-rank bench test, the default bench line, the one-GPU strong-scaling shard curve (C5, C3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_a; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_a] $(date +%T) pytest gather"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_gather.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gather.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gather.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_a] $(date +%T) bench"
timeout -k 10 300 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
cut -c1-400 $OUT/bench_c3.json
echo "[r04_a] $(date +%T) shard curve c5"
timeout -k 10 300 python tools/shard_curve.py --config c5 > $OUT/shard_c5.json 2> $OUT/shard_c5.err || { tail $OUT/shard_c5.err; exit 1; }
cat $OUT/shard_c5.err | grep '^{'
echo "[r04_a] $(date +%T) shard curve c3"
timeout -k 10 300 python tools/shard_curve.py --config c3 > $OUT/shard_c3.json 2> $OUT/shard_c3.err || { tail $OUT/shard_c3.err; exit 1; }
cat $OUT/shard_c3.err | grep '^{'
