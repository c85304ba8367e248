#!/bin/bash
# r04 session AE: the wire decode on 32-bit divisions: wire / gather tests, the exchange parts, the 1-rank exchange lines
# against HEAD (libsvo_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ae; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "wire or exchange or multi_frame or sharding" tests/test_gpu_bench_gather.py tests/test_gpu_bridge.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in base default; do
  if [ $L = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/variants/libsvo_$L.so; fi
  timeout -k 10 300 python tools/xchg_parts.py > $OUT/parts_$L.log 2>&1 || { tail $OUT/parts_$L.log; exit 1; }
  echo "== $L"; cat $OUT/parts_$L.log | grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl"
done
unset SVO_LIB
REPS=4 BENCH_ARGS="--force-exchange --no-cpu-baseline" timeout -k 10 600 bash tools/ab_lib.sh r04_ae/x3 variants/libsvo_base.so default || exit 1
