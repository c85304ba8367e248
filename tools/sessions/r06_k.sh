# r06 session k: the brick walk's one-ahead hint (tools/variants/brickpf.patch): the GPU suite on the
# variant, then A/B against the product on C3, C5 and the shaded frame, and the top-rows probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_k; mkdir -p $O
SVO_LIB=$PWD/variants/libsvo_brickpf.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_brickpf.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/steps.log; tail -3 $O/pytest_brickpf.log
if [ $rc -ne 0 ]; then cat $O/steps.log; exit $rc; fi
REPS=4 bash tools/ab_lib.sh r06_k3 default variants/libsvo_brickpf.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS="--config c5 --steps 20" bash tools/ab_lib.sh r06_k5 default variants/libsvo_brickpf.so > $O/ab_c5.txt 2>&1; echo "ab c5 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_ksh default variants/libsvo_brickpf.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
SVO_LIB=$PWD/variants/libsvo_brickpf.so timeout -k 10 200 python tools/lane_probe.py > $O/lane_brickpf.txt 2>&1; echo "lane rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log; tail -1 $O/lane_brickpf.txt
