#!/bin/bash
# r04 session Q: the refractive pass with the last block's flags cached, without (libsvo_cache) and with (libsvo_sibcache)
# the sibling-brick continuation, against HEAD (libsvo_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_q/ab variants/libsvo_base.so variants/libsvo_cache.so variants/libsvo_sibcache.so || exit 1
