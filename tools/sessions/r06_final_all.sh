# r06 final (one call): the final build's GPU suite and smoke, every config's PMC passes (copied into profiles/ here so
# the bench lines carry same-build counters), tools/evidence.sh, 43-launch kernel traces of C3 and the shaded frame, the
# top-rows probe and the shaded frame's critical path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r06_fa}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so | tee $OUT/lib_sha256.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_all.sh ${TAG}_pmc > $OUT/pmc_all.log 2>&1 || { tail $OUT/pmc_all.log; exit 1; }
for k in c3 c3f c3_ao16 c5 c3_shade c2; do cp gpurun_out/${TAG}_pmc_$k/pmc_summary.json profiles/pmc_$k.json || exit 1; done
bash tools/evidence.sh $TAG/ev > $OUT/evidence.log 2>&1 || { tail -20 $OUT/evidence.log; exit 1; }
tail -8 $OUT/evidence.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_c3.json 2> $OUT/prof_c3.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shade -o run -- python3 bench.py --shade --steps 40 --warmup 3 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_shade.json 2> $OUT/prof_shade.err || exit $?
timeout -k 10 200 python tools/lane_probe.py > $OUT/lane.txt 2>&1 || exit $?
timeout -k 10 300 python tools/shade_critical.py > $OUT/shade_critical.json 2> $OUT/shade_critical.err || exit $?
tail -1 $OUT/lane.txt; cat $OUT/shade_critical.json
