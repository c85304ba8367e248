#!/bin/bash
# r04 session C: the fixed / new GPU tests (pick ray highlight pose, the bench's shaded scene over the whole frame,
# C5 last_pos + material, C4 N = 20 at depth 12), the shading pass's traversal counters, the shaded bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_c; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_c] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py "tests/test_gpu_parity.py::test_depth14_4k_sampled_parity" \
    "tests/test_gpu_parity.py::test_ao_depth12_full_frame" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_c] $(date +%T) shade stats"
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
echo "[r04_c] $(date +%T) shade bench"
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
cut -c1-300 $OUT/bench_shade.json
python -c "import json; d=json.load(open('$OUT/bench_shade.json')); print(json.dumps(d['roofline']))"
