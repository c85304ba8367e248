#!/bin/bash
# The N>1 bench pipeline on one GPU over gloo (2 and 3 ranks, --verify; AO and shaded at 2 ranks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-multi}; mkdir -p $OUT; export TMPDIR=/tmp
run() { local tag=$1; shift; timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }; grep '^{' $OUT/$tag.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['n_gpus'], round(d['value']/1e6,1), 'M rays/s', 'verified', d.get('gather_verified'), d['config'].get('exchange'))"; }
run g2 --nproc-per-node 2 --master-port 29541 bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo --verify
run g3 --nproc-per-node 3 --master-port 29542 bench.py --gpus 3 --steps 6 --warmup 2 --dist-backend gloo --verify
run g2ao --nproc-per-node 2 --master-port 29543 bench.py --gpus 2 --steps 4 --warmup 1 --dist-backend gloo --ao 16 --verify
run g2sh --nproc-per-node 2 --master-port 29544 bench.py --gpus 2 --steps 4 --warmup 1 --dist-backend gloo --shade
