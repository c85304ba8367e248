#!/bin/bash
# r05_r: the march with two blocks of ceiling prefetch (and 1/absDelta set after it) vs HEAD — parity, A/B C3, C4, C5, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_r; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_d2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_shade.py tests/test_gpu_edits.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
V="variants/libsvo_pre2.so variants/libsvo_d2.so"
REPS=3 bash tools/ab_lib.sh r05_r_c3 $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_r_ao $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_r_sh $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_r_c5 $V || exit 1
