#!/bin/bash
# The bench lines of the main configs (after the counters in profiles/ were refreshed).  usage: tools/evidence_lines.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-evl}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
b() { local name=$1; shift; echo "[evidence] $(date +%T) $name"; timeout -k 10 300 python bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_$name.err; exit $rc; }; cut -c1-200 $OUT/bench_$name.json; }
b c3
b c4_ao16 --ao 16
b c4_ao20 --ao 20 --no-cpu-baseline
b c5 --config c5
b c2 --config c2
b c2cam0 --config c2cam0 --no-cpu-baseline
b shade --shade
b c5_xchg1 --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline
