#!/bin/bash
# r04 session O: the working tree (shading bounce state in LDS, 5 waves): the whole GPU suite, shaded bench line with its
# CPU baseline (parity), a rocprofv3 kernel trace of the shaded bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_o; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_o] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shade > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_shade.json')); print(d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'].get('parity_vs_gpu'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shade -o run -- python3 bench.py --shade --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_shade.json 2> $OUT/prof_shade.err || exit 1
grep k_cast $OUT/prof_shade/run_kernel_stats.csv | cut -c1-160
