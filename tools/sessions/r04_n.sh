#!/bin/bash
# r04 session N: bounce state in LDS at 5 (launch bound 8, LDS-limited) vs 6 waves per SIMD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_n/ab variants/libsvo_ldsbn8.so variants/libsvo_w6.so || exit 1
