# r06 session h: the level-1 LDS top cache (SVO_X_TOPC, primary casts of 3-6-level trees): the GPU suite on the
# variant, then A/B against the product on C3, C2 (5 levels) and C5 (7 levels: cache off, a control)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_h; mkdir -p $O
SVO_LIB=$PWD/variants/libsvo_topc.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_topc.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/steps.log; tail -3 $O/pytest_topc.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
REPS=4 bash tools/ab_lib.sh r06_h3 default variants/libsvo_topc.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--config c2" bash tools/ab_lib.sh r06_h2 default variants/libsvo_topc.so > $O/ab_c2.txt 2>&1; echo "ab c2 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--config c5 --steps 20" bash tools/ab_lib.sh r06_h5 default variants/libsvo_topc.so > $O/ab_c5.txt 2>&1; echo "ab c5 rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
