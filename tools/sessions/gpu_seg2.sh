#!/bin/bash
# parity (cast + shade), fractional camera, A/B on the default camera
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-seg}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shade.py tests/test_gpu_edits.py tests/test_gpu_bridge.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --origin 4.37,90.61,4.23 > $OUT/frac.json 2> $OUT/frac.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/frac.json')); print('fractional camera ms', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
shift
REPS=${REPS:-5} bash tools/ab_lib.sh ${OUT#gpurun_out/}_ab "$@"
