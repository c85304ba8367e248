set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/r02a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r02a/pytest.log
exit $rc
