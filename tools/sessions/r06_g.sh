# r06 session g: the root-seeded first parent (SVO_X_ROOT_SEED): the GPU suite on the variant, then A/B against the
# product on C3, shaded C3, C4, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_g; mkdir -p $O
SVO_LIB=$PWD/variants/libsvo_root.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_root.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/steps.log; tail -3 $O/pytest_root.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
REPS=3 bash tools/ab_lib.sh r06_g3 default variants/libsvo_root.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=3 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_gsh default variants/libsvo_root.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r06_g4 default variants/libsvo_root.so > $O/ab_c4.txt 2>&1; echo "ab c4 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--config c5 --steps 20" bash tools/ab_lib.sh r06_g5 default variants/libsvo_root.so > $O/ab_c5.txt 2>&1; echo "ab c5 rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
