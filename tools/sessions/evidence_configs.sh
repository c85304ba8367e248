#!/bin/bash
# Kernel traces and PMC traffic of the other configs (C5, C4, shaded): tools/evidence_configs.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-evc}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1; shift; echo "[evidence] $(date +%T) $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step c5_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_prof.json 2> $OUT/c5.err
step c4_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --ao 16 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_prof.json 2> $OUT/c4.err
step shade_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shade -o run -- python3 bench.py --shade --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_shade_prof.json 2> $OUT/shade.err
step c5_pmc timeout -k 10 900 bash tools/pmc.sh ${TAG}_c5_pmc --config c5
