# r06 session c: the GPU suite on the candidate product library, then A/B against the round's base (variants/libsvo_base6.so:
# dispatch table only) on C3, shaded C3, C4 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/steps.log
tail -3 $O/pytest_gpu.log
if [ $rc -ge 124 ]; then exit $rc; fi
REPS=3 bash tools/ab_lib.sh r06_c3 default variants/libsvo_base6.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=3 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_sh default variants/libsvo_base6.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--config c5 --steps 20" bash tools/ab_lib.sh r06_c5 default variants/libsvo_base6.so > $O/ab_c5.txt 2>&1; echo "ab c5 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r06_c4 default variants/libsvo_base6.so > $O/ab_c4.txt 2>&1; echo "ab c4 rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
