#!/bin/bash
# r04 session AP: the exchange's decode in 512- and 1024-thread blocks (held back to the next cast's tail) against 256
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--force-exchange" timeout -k 10 600 bash tools/ab_lib.sh r04_ap/c3 variants/libsvo_base.so variants/libsvo_sc512.so variants/libsvo_sc1024.so || exit 1
