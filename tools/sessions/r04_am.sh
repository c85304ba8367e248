#!/bin/bash
# r04 session AM: is the 1-rank exchange step host-bound? (tools/xchg_host.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_am; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/xchg_host.py > $OUT/host.log 2>&1; rc=$?; grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids" $OUT/host.log; exit $rc
