#!/bin/bash
# One guarded GPU session: gpu tests -> bench -> rocprofv3 kernel trace.  Stops at the first step that
# crashes, aborts or times out (rc >= 124 or a signal); ordinary test failures (rc 1) continue.
# usage: tools/gpu_round.sh [tag] [pytest-args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }

echo "[gpu_round] $(date) pytest" | tee -a "$OUT/steps.log"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.log"; tail -5 "$OUT/pytest_gpu.log"
if fatal $rc; then exit $rc; fi

echo "[gpu_round] $(date) bench" | tee -a "$OUT/steps.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if [ $rc -ne 0 ]; then exit $rc; fi

echo "[gpu_round] $(date) rocprofv3 kernel trace" | tee -a "$OUT/steps.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/steps.log"
find "$OUT/prof" -name "*stats*" | head
exit $rc
