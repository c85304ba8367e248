#!/bin/bash
# r04 session AU: shading-only frame schedules: schedule + shading GPU tests, shaded bench line, its kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_au; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_shade.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['config']['dispatch_order'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; cut -c1-200 $OUT/kernel_stats_shade.csv | head -8
