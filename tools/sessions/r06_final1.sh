# r06 final, part 1: the final build's GPU suite, smoke, and every config's PMC passes (summaries under
# gpurun_out/r06_pmc_<config>/, copied to profiles/pmc_<config>.json before part 2 takes the bench lines)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06_final1; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so | tee $OUT/lib_sha256.txt
echo "[r06_final1] $(date +%T) pytest"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_all.sh r06_pmc || exit $?
