#!/bin/bash
# r04 session AZ: the schedule by groups of 4 blocks (a quarter of the sort): schedule tests, shaded bench line, its
# kernel trace (k_sched_order's duration), and the schedule under camera motion (tools/shade_motion.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_az; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; grep -E "k_cast|k_sched" $OUT/kernel_stats_shade.csv | cut -d, -f2-4 
timeout -k 10 400 python tools/shade_motion.py 40 > $OUT/motion.log 2> $OUT/motion.err || { tail $OUT/motion.err; exit 1; }
cat $OUT/motion.log
