set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "shade or build or bridge or edits" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shade > $OUT/bench_shade.json 2> $OUT/bench_shade.err; rc=$?; echo "shade rc=$rc"; cut -c1-600 $OUT/bench_shade.json
