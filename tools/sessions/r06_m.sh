# r06 session m: the AO plan's bricks looked up two at a time (tools/variants/aopair.patch): the AO parity tests on the
# variant, then A/B against the product on C4 (16 and 20 AO rays)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_m; mkdir -p $O
SVO_LIB=$PWD/variants/libsvo_aopair.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "ao" > $O/pytest_aopair.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/steps.log; tail -2 $O/pytest_aopair.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
REPS=4 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r06_m4 default variants/libsvo_aopair.so > $O/ab_c4.txt 2>&1; echo "ab c4 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--ao 20" bash tools/ab_lib.sh r06_m20 default variants/libsvo_aopair.so > $O/ab_c4_20.txt 2>&1; echo "ab c4_20 rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
