# r06 session d: which of the two register changes slowed C3 (x<reload><iter-regs>: reload = the origin re-read after the
# trace; iter-regs 1 = brick registers zeroed per iteration, 2 = per iteration without a value); default = x11
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_d; mkdir -p $O
REPS=3 bash tools/ab_lib.sh r06_d3 default variants/libsvo_base6.so variants/libsvo_x00.so variants/libsvo_x10.so variants/libsvo_x01.so variants/libsvo_x12.so variants/libsvo_x02.so > $O/ab_c3.txt 2>&1; echo "ab c3 rc=$?" >> $O/steps.log
REPS=2 BENCH_ARGS=--shade bash tools/ab_lib.sh r06_dsh default variants/libsvo_x00.so variants/libsvo_x12.so variants/libsvo_x02.so > $O/ab_shade.txt 2>&1; echo "ab shade rc=$?" >> $O/steps.log
cat $O/ab_*.txt $O/steps.log
