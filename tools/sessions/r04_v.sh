#!/bin/bash
# r04 session V: the non-segment shading instance (test + A/B), and the C3 critical path (one-GPU shard curve, N = 1 / 8)
# of the per-level ceiling quads (libsvo_quadprim) against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_v; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/sessions/r04_u.sh || exit 1
for L in base quadprim; do
  SVO_LIB=$PWD/variants/libsvo_$L.so timeout -k 10 300 python tools/shard_curve.py --config c3 --ns 1,8 > $OUT/shard_$L.json 2> $OUT/shard_$L.err || { tail $OUT/shard_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/shard_$L.json')); print('$L', [(r['n'], r['max_us'], round(sum(r['rank_us'])/len(r['rank_us']),1), r['inflight_max_us']) for r in d['curve']])"
done
