# r06 session i: two-block ceiling boxes (tools/variants/ceil2.patch, SVO_X_CEIL2): the GPU suite on the variant, then
# A/B against the product on C3, C5, C4 and the shaded frame; the AO brick-record prefetch (tools/variants/aopf.patch) on C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_i; mkdir -p $O
SVO_LIB=$PWD/variants/libsvo_ceil2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_ceil2.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/steps.log; tail -3 $O/pytest_ceil2.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
SVO_LIB=$PWD/variants/libsvo_aopf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "ao" > $O/pytest_aopf.log 2>&1; rc=$?; echo "pytest aopf rc=$rc" >> $O/steps.log; tail -2 $O/pytest_aopf.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
REPS=4 bash tools/ab_lib.sh r06_i3 default variants/libsvo_ceil2.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--config c5 --steps 20" bash tools/ab_lib.sh r06_i5 default variants/libsvo_ceil2.so > $O/ab_c5.txt 2>&1; echo "ab c5 rc=$?" >> $O/steps.log
REPS=3 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r06_i4 default variants/libsvo_ceil2.so variants/libsvo_aopf.so > $O/ab_c4.txt 2>&1; echo "ab c4 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_ish default variants/libsvo_ceil2.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
SVO_LIB=$PWD/variants/libsvo_ceil2.so timeout -k 10 200 python tools/lane_probe.py > $O/lane_ceil2.txt 2>&1; echo "lane rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log; tail -1 $O/lane_ceil2.txt
