#!/bin/bash
# r05_b: the bridge (main.cpp-shaped TU) and the N > 1 C-ABI exchange through the RCCL stand-in, on one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bridge.py tests/test_gpu_bench_gather.py > $OUT/pytest.log 2>&1
rc=$?; tail -30 $OUT/pytest.log; exit $rc
