#!/bin/bash
# r04 session B: the shading pass's traversal counters (STATS instance), the shaded bench line, the edits tests
# (incremental device ceilings), the C3 full frame (guard counter), the shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_b; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_b] $(date +%T) shade stats"
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
echo "[r04_b] $(date +%T) shade bench"
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
cut -c1-300 $OUT/bench_shade.json
echo "[r04_b] $(date +%T) bench c3"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail $OUT/bench_c3.err; exit 1; }
cut -c1-300 $OUT/bench_c3.json
echo "[r04_b] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_edits.py tests/test_gpu_shade.py "tests/test_gpu_parity.py::test_depth12_full_frame_parity" -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
grep -E "edit \+ sync|passed|failed" $OUT/pytest.log | tail -5; exit $rc
