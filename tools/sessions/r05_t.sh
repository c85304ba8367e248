#!/bin/bash
# r05_t: REFLECT sign flags re-derived only after a bounce (flags); + shading launches without hit records keep no
# crossing value (norec) — shading parity, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_t; mkdir -p $OUT
for v in flags norec; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest_$v.log 2>&1
rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_$v.log | head -20; exit $rc; }
done
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_t_sh variants/libsvo_pre2.so variants/libsvo_flags.so variants/libsvo_norec.so || exit 1
