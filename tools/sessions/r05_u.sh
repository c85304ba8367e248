#!/bin/bash
# r05_u: shading launches without hit records keep no crossing value (norec2, on HEAD); diagnostic: the shading trace
# without the reflection / refraction machinery (norefl: wrong images, timing only) — parity of norec2, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_u; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_norec2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_u_sh variants/libsvo_pre2.so variants/libsvo_norec2.so variants/libsvo_norefl.so || exit 1
