#!/bin/bash
# r05_f: A/B of the column-ceiling granularity: 4-column finest level (SVO_CEIL_K0 1; primary pairs 4/16 or 4/64)
# against the shipped 16/64 — C3, C5, shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=3 bash tools/ab_lib.sh r05_f_c3 default variants/libsvo_k01.so variants/libsvo_k01p02.so || exit 1
REPS=2 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_f_c5 default variants/libsvo_k01.so variants/libsvo_k01p02.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_f_sh default variants/libsvo_k01.so variants/libsvo_k01p02.so || exit 1
