#!/bin/bash
# r04 session BH: C5's block timeline (bench.py --stats with SVO_STAMPS) — is the 4K launch bound by its longest waves?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_bh; mkdir -p $OUT; export TMPDIR=/tmp
SVO_STAMPS=$OUT/stamps_c5.npy timeout -k 10 300 python bench.py --config c5 --stats --steps 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5_stats.err || { tail $OUT/c5_stats.err; exit 1; }
tail -25 $OUT/c5_stats.err
