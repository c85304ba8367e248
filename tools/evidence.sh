#!/bin/bash
# One guarded evidence session (after the GPU parity suite has passed): bench lines of every config
# (C3 / C4 / C5 / C2 / shaded with their CPU baselines, C1), the single-rank C-ABI RCCL exchange, gloo
# rehearsals of the N>1 paths on one GPU (weak, strong, AO, shaded), the C-ABI exchange at N = 2, 3 over the
# test-only RCCL stand-in, the rocprofv3 kernel traces.  usage: tools/evidence.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ev}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1; shift; echo "[evidence] $(date +%T) $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
b() { local name=$1; shift; echo "[evidence] $(date +%T) $name"; timeout -k 10 300 python bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_$name.err; exit $rc; }; cut -c1-300 $OUT/bench_$name.json; }
d() { local name=$1 n=$2 port=$3; shift 3; echo "[evidence] $(date +%T) $name"; timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --dist-backend gloo "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_$name.err; exit $rc; }; grep '^{' $OUT/bench_$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['n_gpus'], d['scaling'], round(d['value']/1e6,1), 'M rays/s', 'verified', d.get('gather_verified'))"; }
# the C-ABI exchange at N > 1 (svo_cast_wire + svo_exchange_wire, ncclGroupStart/Send/Recv/GroupEnd) with N ranks on
# this one GPU: libsvo_rt dlopens the TEST-ONLY host-staged stand-in (SVO_RCCL_LIB) in place of RCCL, which cannot form a
# communicator of N ranks on one device; bench.py verifies the displayed frames at N > 1 by default
s() { local name=$1 n=$2; shift 2; echo "[evidence] $(date +%T) $name"; mkdir -p $OUT/standin_$name; SVO_RCCL_LIB=$PWD/tests/standin/_build/librccl_standin.so SVO_RCCL_STANDIN=1 SVO_STANDIN_DIR=$OUT/standin_$name SVO_STANDIN_TIMEOUT_S=60 timeout -k 10 300 python bench.py --gpus $n --dist-backend gloo --exchange capi --no-cpu-baseline "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_$name.err; exit $rc; }; grep '^{' $OUT/bench_$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['n_gpus'], d['scaling'], round(d['value']/1e6,1), 'M rays/s', 'verified', d.get('gather_verified'))"; }
b c3
b c3f --config c3f
b c1 --config c1
b c4_ao16 --ao 16
b c4_ao20 --ao 20 --no-cpu-baseline
b c5 --config c5
b c2 --config c2
b c2cam0 --config c2cam0 --no-cpu-baseline
b c2d8 --config c2d8
b shade --shade
b xchg1 --force-exchange --verify --no-cpu-baseline
b xchg1_ao --force-exchange --verify --no-cpu-baseline --ao 16
b c5_xchg1 --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline
d g2 2 29541 --steps 4 --warmup 1 --verify
d g2_strong 2 29542 --steps 4 --warmup 1 --frames 1 --verify
d g3_f2 3 29543 --steps 4 --warmup 1 --frames 2 --verify
d g2_ao 2 29544 --steps 4 --warmup 1 --ao 16 --verify
d g2_shade 2 29545 --steps 4 --warmup 1 --shade
d g2_strong_if2 2 29546 --steps 4 --warmup 1 --frames 1 --inflight 2 --verify
b c5_if2 --config c5 --frames 1 --inflight 2 --no-cpu-baseline
s g2_capi 2 --steps 4 --warmup 1
s g3_capi 3 --steps 4 --warmup 1
s g2_capi_strong 2 --steps 4 --warmup 1 --frames 1
s g3_capi_strong_ao 3 --steps 4 --warmup 1 --frames 1 --ao 16
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof.json 2> $OUT/prof.err
step rocprof_c5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_c5.json 2> $OUT/prof_c5.err
step rocprof_c4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --ao 16 --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_c4.json 2> $OUT/prof_c4.err
step rocprof_c3f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3f -o run -- python3 bench.py --config c3f --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_c3f.json 2> $OUT/prof_c3f.err
step rocprof_shade timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shade -o run -- python3 bench.py --shade --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_shade.json 2> $OUT/prof_shade.err
