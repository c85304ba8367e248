# r06 session b: A/B of the in-loop march variants (C3), the sun-octant shadow rays (shaded C3), then C3-frame parity of
# the 8-wave march variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_b; mkdir -p $O
REPS=3 bash tools/ab_lib.sh r06_b default variants/libsvo_im1.so variants/libsvo_im2.so variants/libsvo_im1w7.so variants/libsvo_im2w7.so > $O/ab.txt 2>&1; echo "ab rc=$?" >> $O/steps.log
cat $O/ab.txt
REPS=3 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_b_sh default variants/libsvo_sun.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
cat $O/ab_shade.txt
for v in im1 im2; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "depth12 or c3" > $O/parity_$v.log 2>&1; echo "parity $v rc=$?" >> $O/steps.log; tail -2 $O/parity_$v.log
done
cat $O/steps.log
