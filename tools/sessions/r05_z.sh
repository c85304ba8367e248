#!/bin/bash
# r05_z: the ceiling march takes the parent block's ceiling (no load) for the blocks inside a parent the ray stays above
# (pmarch) — full GPU suite on it, A/B C3 / C4 / C5 / shaded against the HEAD build (h9f)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_z; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_pmarch.so timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 bash tools/ab_lib.sh r05_z_c3 variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_z_ao variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r05_z_c5 variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_z_sh variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
