#!/bin/bash
# r05_h: column-ceiling layouts with the pair table's partner level configurable (SVO_CEIL_PAIR_STEP): finest level
# 4 or 16 columns (SVO_CEIL_K0 1 / 2), second level 2 or 3 levels up — parity of each variant (the whole C3 frame, the
# edits' tables), then A/B C3, C5, C4, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_h; mkdir -p $OUT
for v in k1s2 k1s3 k2s2 k2s3; do
  SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_edits.py tests/test_gpu_small_trees.py -k "depth12 or edits or small or ceiling or frame" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ge 124 ] && exit $rc
done
V="default variants/libsvo_k1s2.so variants/libsvo_k1s3.so variants/libsvo_k2s2.so variants/libsvo_k2s3.so"
REPS=3 bash tools/ab_lib.sh r05_h_c3 $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_h_sh $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_h_ao $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_h_c5 $V || exit 1
