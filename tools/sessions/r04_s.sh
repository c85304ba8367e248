#!/bin/bash
# r04 session S: ceiling boxes chosen by latest exit among every level the ray is above (f32 estimate): primary casts
# (libsvo_quadlate) against the 16/64 pair (HEAD) and the coarsest level (libsvo_quadprim); the shading pass (libsvo_shadelate)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_s/c3 variants/libsvo_base.so variants/libsvo_quadlate.so || exit 1
REPS=3 BENCH_ARGS="--config c5" timeout -k 10 600 bash tools/ab_lib.sh r04_s/c5 variants/libsvo_base.so variants/libsvo_quadlate.so || exit 1
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_s/shade variants/libsvo_base.so variants/libsvo_shadelate.so || exit 1
