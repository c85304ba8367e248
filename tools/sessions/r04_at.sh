#!/bin/bash
# r04 session AT: frame schedules (longest block first from the last frame): parity, then A/B against the default order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_at; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
REPS=3 BENCH_ARGS="--shade" bash tools/ab_flags.sh r04_at/shade 0 65536 || exit 1
REPS=3 bash tools/ab_flags.sh r04_at/c3 0 65536 || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_flags.sh r04_at/c5 0 65536 || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_flags.sh r04_at/c4 0 65536 || exit 1
timeout -k 10 300 python tools/shade_timeline.py $OUT/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || exit 1
cut -c1-600 $OUT/timeline.json
