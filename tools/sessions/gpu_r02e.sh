set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --stats --no-cpu-baseline > $OUT/bench_stats.json 2> $OUT/bench_stats.err; rc=$?; echo "stats rc=$rc"; grep -E "stats|timeline" $OUT/bench_stats.err | cut -c1-1500
