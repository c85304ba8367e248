#!/bin/bash
# r04 session R: primary casts walking every ceiling level (max-mipmap quads, CEIL 2) against the 16/64 pair (HEAD): C3, C5, C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_r/c3 variants/libsvo_base.so variants/libsvo_quadprim.so || exit 1
REPS=3 BENCH_ARGS="--config c5" timeout -k 10 600 bash tools/ab_lib.sh r04_r/c5 variants/libsvo_base.so variants/libsvo_quadprim.so || exit 1
REPS=3 BENCH_ARGS="--ao 16" timeout -k 10 600 bash tools/ab_lib.sh r04_r/c4 variants/libsvo_base.so variants/libsvo_quadprim.so || exit 1
