#!/bin/bash
# r04 session AA: shading with the ceiling quads' coarse levels only after a reflection / refraction (the 16 / 64 choice
# before), against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=5 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_aa/ab variants/libsvo_base.so variants/libsvo_turned.so || exit 1
