set -o pipefail
O=gpurun_out/r06_a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_gather.py -x -v --timeout 250 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/steps.log
timeout -k 10 300 python bench.py --no-c1 > $O/c3.json 2> $O/c3.err && echo "c3 ok" >> $O/steps.log && \
timeout -k 10 200 python bench.py --no-cpu-baseline --shade > $O/shade.json 2> $O/shade.err && echo "shade ok" >> $O/steps.log && \
timeout -k 10 200 python tools/lane_probe.py > $O/lane.txt 2>&1; echo "lane rc=$?" >> $O/steps.log
cat $O/steps.log; tail -5 $O/pytest.log
