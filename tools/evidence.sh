#!/bin/bash
# One guarded evidence session (after the GPU parity suite has passed): bench lines for C3 (+ CPU
# baseline), C4 (16 / 20 AO rays), C5 and the shading pass, a 2-rank gloo rehearsal of the N>1 path on
# one GPU, the rocprofv3 kernel trace of the C3 bench, then the PMC passes (traffic, SQ).
# usage: tools/evidence.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ev}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1; shift; echo "[evidence] $(date +%T) $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step c3 timeout -k 10 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step c4_16 timeout -k 10 120 bash -c "python bench.py --ao 16 --no-cpu-baseline > $OUT/bench_c4_ao16.json 2>> $OUT/bench.err"
step c4_20 timeout -k 10 120 bash -c "python bench.py --ao 20 --no-cpu-baseline > $OUT/bench_c4_ao20.json 2>> $OUT/bench.err"
step c5 timeout -k 10 300 bash -c "python bench.py --config c5 > $OUT/bench_c5.json 2>> $OUT/bench.err"
step c2 timeout -k 10 120 bash -c "python bench.py --config c2 --no-cpu-baseline > $OUT/bench_c2.json 2>> $OUT/bench.err"
step c2cam0 timeout -k 10 120 bash -c "python bench.py --config c2cam0 --no-cpu-baseline > $OUT/bench_c2cam0.json 2>> $OUT/bench.err"
step shade timeout -k 10 120 bash -c "python bench.py --shade --no-cpu-baseline > $OUT/bench_shade.json 2>> $OUT/bench.err"
step gloo2 timeout -k 10 300 bash -c "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --verify > $OUT/bench_gloo2.json 2> $OUT/gloo2.err"
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err
step pmc timeout -k 10 600 bash tools/pmc.sh ${TAG}_pmc
step sq timeout -k 10 600 bash tools/pmc_sq.sh ${TAG}_sq
