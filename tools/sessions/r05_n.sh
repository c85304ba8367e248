#!/bin/bash
# r05_n: 1/absDelta recomputed per use (Ray.ia dropped: no spill with the march) vs the march commit — parity, A/B C3, C4,
# C5, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_n; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_noia.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_shade.py > $OUT/pytest.log 2>&1
SVO_LIB=$PWD/variants/libsvo_shmarch.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest_sh.log 2>&1; rc2=$?; echo "shmarch pytest rc=$rc2: $(tail -1 $OUT/pytest_sh.log)"
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_n_c3 variants/libsvo_pre.so variants/libsvo_noia.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_n_ao variants/libsvo_pre.so variants/libsvo_noia.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_n_sh variants/libsvo_pre.so variants/libsvo_noia.so variants/libsvo_shmarch.so || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_n_c5 variants/libsvo_pre.so variants/libsvo_noia.so || exit 1
