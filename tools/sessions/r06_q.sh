# r06 session q: LLVM machine-scheduler strategies for the whole library (tools/build_variant.py --flag): max-ilp and
# iterative-ilp against the default on C3 and the shaded frame
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_q; mkdir -p $O
SVO_LIB=$PWD/variants/libsvo_iglp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "depth12_full_frame_parity or octant" > $O/pytest_iglp.log 2>&1; rc=$?; echo "pytest iglp rc=$rc" >> $O/steps.log; tail -2 $O/pytest_iglp.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
REPS=4 bash tools/ab_lib.sh r06_q3 default variants/libsvo_milp.so variants/libsvo_iglp.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_qsh default variants/libsvo_milp.so variants/libsvo_iglp.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
