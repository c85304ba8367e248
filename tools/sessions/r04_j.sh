#!/bin/bash
# r04 session J: split shading (two passes): shading tests, then the shaded frame split (default) against one pass
# (--shade-passes 1) and HEAD's single pass (libsvo_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_j; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_j] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade --shade-passes 1" timeout -k 10 600 bash tools/ab_lib.sh r04_j/ab1 variants/libsvo_base.so default || exit 1
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_j/ab2 default || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --shade --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
cut -c1-120 $OUT/prof/run_kernel_stats.csv | head -8
