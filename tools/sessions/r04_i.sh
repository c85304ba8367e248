#!/bin/bash
# r04 session I: the whole GPU suite on the working tree, then the shaded bench line with its CPU baseline (parity)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_i; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_i] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shade > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_shade.json')); print(d['ms_per_step'], json.dumps(d['roofline'])[:300], d['cpu_baseline'].get('parity_vs_gpu'))"
