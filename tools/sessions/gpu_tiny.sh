set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/tiny
echo "== HEAD library (expected to fail before the fix)"
SVO_LIB=$PWD/variants/libsvo_base2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k tiny -x -q --timeout 120 --timeout-method thread > gpurun_out/tiny/head.log 2>&1; echo "head rc=$?"; grep -E "passed|failed|Error" gpurun_out/tiny/head.log | tail -3
for L in fix2; do
SVO_LIB=$PWD/variants/libsvo_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tiny or edge or random or fractional or octant" -x -q --timeout 120 --timeout-method thread > gpurun_out/tiny/$L.log 2>&1; rc=$?; echo "$L rc=$rc"; tail -2 gpurun_out/tiny/$L.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
REPS=4 timeout -k 10 900 bash tools/ab_lib.sh tinyab variants/libsvo_base2.so variants/libsvo_fix2.so
