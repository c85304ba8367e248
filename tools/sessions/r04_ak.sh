#!/bin/bash
# r04 session AK: gloo rehearsals of more ranks on one GPU — weak C3 at N = 4 and 6, strong C5 (one 4K frame) at N = 4 with
# two frames in flight; every displayed frame verified against a one-GPU cast
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ak; mkdir -p $OUT; export TMPDIR=/tmp
d() { local name=$1 n=$2 port=$3; shift 3; echo "[ak] $(date +%T) $name"; timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --dist-backend gloo "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$name.err; exit $rc; }; grep '^{' $OUT/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['n_gpus'], d['scaling'], round(d['value']/1e6,1), 'M rays/s', 'verified', d.get('gather_verified'))"; }
d g4_weak 4 29651 --steps 4 --warmup 1 --verify
d g6_weak 6 29652 --steps 3 --warmup 1 --verify
d g4_c5_strong_if2 4 29653 --config c5 --frames 1 --inflight 2 --steps 4 --warmup 1 --verify
# the 1-rank exchange's kernels (C3): the fused cast and the decode, from a kernel trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_x1 -o run -- python3 bench.py --force-exchange --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_x1.json 2> $OUT/prof_x1.err || exit 1
cut -c1-150 $OUT/prof_x1/run_kernel_stats.csv | head -6
