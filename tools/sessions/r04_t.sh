#!/bin/bash
# r04 session T: primary casts on the per-level ceiling quads, shallow rays (a_y > K min(a_x, a_z)) taking the coarsest
# block they are above and the others the 16/64 pair's choice: K = 4, 10, against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_t/c3 variants/libsvo_base.so variants/libsvo_hyb4.so variants/libsvo_hyb10.so || exit 1
REPS=3 BENCH_ARGS="--config c5" timeout -k 10 600 bash tools/ab_lib.sh r04_t/c5 variants/libsvo_base.so variants/libsvo_hyb4.so variants/libsvo_hyb10.so || exit 1
