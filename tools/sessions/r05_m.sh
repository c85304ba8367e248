#!/bin/bash
# r05_m: the march inside the loop too (every ceiling move of a descending ray marches on) vs the pre-loop march only:
# parity of the in-loop build, then A/B C3, C4, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_m; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_inloop.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_edits.py tests/test_gpu_large.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_m_c3 variants/libsvo_pre.so variants/libsvo_inloop.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_m_ao variants/libsvo_pre.so variants/libsvo_inloop.so || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_m_c5 variants/libsvo_pre.so variants/libsvo_inloop.so || exit 1
