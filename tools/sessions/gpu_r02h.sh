set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py tests/test_gpu_bridge.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shade > $OUT/bench_shade.json 2> $OUT/bench_shade.err; rc=$?; echo "shade rc=$rc"; cut -c1-300 $OUT/bench_shade.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?; echo "c3 rc=$rc"; cut -c1-300 $OUT/bench_c3.json
