#!/bin/bash
# r05_g: column-ceiling granularity, second A/B: primary pairs 4/64 (k01p02), 4/256 (k1p03), shadow pairs 4/64 (k1p02s02),
# 1-column finest level (k0p03: 1/64, k0p13: 4/64) — C3, C5, shaded C3, C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
V="default variants/libsvo_k01p02.so variants/libsvo_k1p03.so variants/libsvo_k1p02s02.so variants/libsvo_k0p03.so variants/libsvo_k0p13.so"
REPS=3 bash tools/ab_lib.sh r05_g_c3 $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_g_sh $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_g_ao $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_g_c5 default variants/libsvo_k01p02.so variants/libsvo_k1p03.so || exit 1
