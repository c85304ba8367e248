# r06 session p: AO brick groups at lower occupancy (tools/variants/aogroup_waves.patch: 2 bricks at 7 waves, 3 at 6):
# the AO parity tests on both, A/B against the product (pairs at 8 waves) on C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_p; mkdir -p $O
for v in aog2w7 aog3w6; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_trees.py -x -q --timeout 250 --timeout-method thread -k "ao" > $O/pytest_$v.log 2>&1; rc=$?; echo "pytest $v rc=$rc" >> $O/steps.log; tail -2 $O/pytest_$v.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
done
REPS=4 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r06_p4 default variants/libsvo_aog2w7.so variants/libsvo_aog3w6.so > $O/ab_c4.txt 2>&1; echo "ab c4 rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
