set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v16; export TMPDIR=/tmp
rc=0
tail -3 gpurun_out/v16/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/v16/b1.json 2>gpurun_out/v16/b1.err || exit 1
tail -c 400 gpurun_out/v16/b1.json
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 6 --warmup 2 --dist-backend gloo --verify > gpurun_out/v16/g$n.json 2> gpurun_out/v16/g$n.err || { tail -20 gpurun_out/v16/g$n.err; exit 1; }
  grep -o '"gather_verified.*' gpurun_out/v16/g$n.json
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 4 --warmup 1 --dist-backend gloo --shade > gpurun_out/v16/g2s.json 2> gpurun_out/v16/g2s.err || { tail -20 gpurun_out/v16/g2s.err; exit 1; }
grep '^{' gpurun_out/v16/g2s.json | cut -c1-200
