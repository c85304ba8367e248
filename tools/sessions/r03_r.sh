#!/bin/bash
# r03 session R: bench.py's torch-exchange gather with the packed wire stride (weak-mode frames verify again): the new
# gpu test, then the gloo rehearsals of tools/evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_r; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r03_r] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
d() { local name=$1 n=$2 port=$3; shift 3; echo "[r03_r] $(date +%T) $name"; timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --dist-backend gloo "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_$name.err; exit $rc; }; grep '^{' $OUT/bench_$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['n_gpus'], d['scaling'], round(d['value']/1e6,1), 'M rays/s', 'verified', d.get('gather_verified'))"; }
d g2 2 29541 --steps 4 --warmup 1 --verify
d g2_strong 2 29542 --steps 4 --warmup 1 --frames 1 --verify
d g3_f2 3 29543 --steps 4 --warmup 1 --frames 2 --verify
d g2_ao 2 29544 --steps 4 --warmup 1 --ao 16 --verify
d g2_shade 2 29545 --steps 4 --warmup 1 --shade
d g4_c3f 4 29546 --steps 4 --warmup 1 --config c3f --verify
