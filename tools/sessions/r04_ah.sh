#!/bin/bash
# r04 session AH: occupancy sensitivity of the primary instance: 5 and 6 waves per SIMD against 8 (C3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=3 timeout -k 10 600 bash tools/ab_lib.sh r04_ah/c3 variants/libsvo_base.so variants/libsvo_prim5.so variants/libsvo_prim6.so || exit 1
