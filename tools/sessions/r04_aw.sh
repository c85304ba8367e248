#!/bin/bash
# r04 session AW: block timelines with the shading schedule (primary in its default order); shading waves per SIMD
# under the schedule (4 / 5 / 6, variants built by tools/build_variant.py --patch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_aw; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_timeline.py $OUT/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
cut -c1-300 $OUT/timeline.json
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r04_aw/shade default variants/libsvo_shade_w4.so variants/libsvo_shade_w6.so
