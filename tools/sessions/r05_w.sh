#!/bin/bash
# r05_w: the straight trace of shading rays on the camera's step octant (cam; shadow rays then take generic sign flags),
# the same at 6 waves per SIMD (cam6) — shading parity, A/B shaded C3 against split (r05_v) and HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_w; mkdir -p $OUT
for v in cam cam6; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest_$v.log 2>&1
rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_$v.log | head -20; exit $rc; }
done
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_w_sh variants/libsvo_norec2.so variants/libsvo_split.so variants/libsvo_cam.so variants/libsvo_cam6.so || exit 1
