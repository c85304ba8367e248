#!/bin/bash
# r05_aa: where the C3 critical path stands after the ceiling march: per-wave work of the longest waves (STATS build
# stamps + per-ray work), the shard curve (N = 1..8, one launch at a time and in flight)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_aa; mkdir -p $OUT
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/bench.json 2> $OUT/bench.err || exit 1
python tools/wave_work.py $OUT/stamps.npy $OUT/work.npy > $OUT/wave_work.txt 2>&1; echo "wave_work rc=$?"
timeout -k 10 300 python tools/shard_curve.py --config c3 > $OUT/shard_c3.json 2> $OUT/shard_c3.err || exit 1
timeout -k 10 300 python tools/shard_curve.py --config c5 > $OUT/shard_c5.json 2> $OUT/shard_c5.err || exit 1
head -30 $OUT/wave_work.txt
python3 -c "
import json
for c in ('c3','c5'):
    d=json.loads([l for l in open('$OUT/shard_%s.json'%c) if l.startswith('{')][-1])
    for e in d['curve']: print(c, e['n'], e['max_us'], e['ideal_us'], e.get('inflight_max_us'), e['rank_us'])"
