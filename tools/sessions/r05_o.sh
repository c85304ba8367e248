#!/bin/bash
# r05_o: the march in the shading trace too (stored 1/absDelta kept) — the whole GPU suite, then A/B shaded / C3 vs the
# march commit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_o; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_o_sh variants/libsvo_pre.so default || exit 1
REPS=3 bash tools/ab_lib.sh r05_o_c3 variants/libsvo_pre.so default || exit 1
