# r06 session n: the AO plan's bricks in groups with slim per-brick state (tools/variants/aoslim.patch, groups of 2 and
# 3): the AO parity tests on both, then A/B against the product (bricks in pairs) on C4 (16 and 20 AO rays)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_n; mkdir -p $O
for v in aoslim2 aoslim3; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_trees.py -x -q --timeout 250 --timeout-method thread -k "ao" > $O/pytest_$v.log 2>&1; rc=$?; echo "pytest $v rc=$rc" >> $O/steps.log; tail -2 $O/pytest_$v.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
done
REPS=4 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r06_n4 default variants/libsvo_aoslim2.so variants/libsvo_aoslim3.so > $O/ab_c4.txt 2>&1; echo "ab c4 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--ao 20" bash tools/ab_lib.sh r06_n20 default variants/libsvo_aoslim2.so variants/libsvo_aoslim3.so > $O/ab_c4_20.txt 2>&1; echo "ab c4_20 rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
