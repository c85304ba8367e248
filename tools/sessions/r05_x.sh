#!/bin/bash
# r05_x: the straight shading trace on the launch's two ceiling levels (cam1: CEIL 1, as primary casts) instead of
# the walk over every level (cam6: CEIL 2) — shading parity, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_x; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_cam1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_x_sh variants/libsvo_cam6.so variants/libsvo_cam1.so || exit 1
