#!/bin/bash
# r04 session AQ: the 1024-thread decode: wire / exchange / gather / bridge tests, the forced 1-rank exchange lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_aq; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "wire or exchange or multi_frame or sharding" tests/test_gpu_bench_gather.py tests/test_gpu_bridge.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in "xchg1 --force-exchange --verify" "xchg1_ao --force-exchange --verify --ao 16" "c5_xchg1 --config c5 --frames 1 --force-exchange --verify"; do
  set -- $c; name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  grep '^{' $OUT/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], round(d['value']/1e9,2), d.get('gather_verified'))"
done
