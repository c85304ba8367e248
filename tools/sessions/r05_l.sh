#!/bin/bash
# r05_l: the column-ceiling march (ceil_march) — parity (parity, configs, small trees, edits, large, AO), then A/B against
# the round's previous commit (variants/libsvo_base.so): C3, C4, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_edits.py tests/test_gpu_large.py tests/test_gpu_build.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_l_c3 variants/libsvo_base.so default || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_l_ao variants/libsvo_base.so default || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_l_c5 variants/libsvo_base.so default || exit 1
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/stats.json 2> $OUT/stats.txt
grep "stats per ray" $OUT/stats.txt | head -2
