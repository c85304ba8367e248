# r06 final, part 3: longer rocprofv3 kernel traces of C3 and the shaded frame (40 timed launches, so the traced
# process's cold first launch weighs 1/45 of the average), the top-rows probe and the shaded frame's critical path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06_final3; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_c3.json 2> $OUT/prof_c3.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shade -o run -- python3 bench.py --shade --steps 40 --warmup 3 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_shade.json 2> $OUT/prof_shade.err || exit $?
timeout -k 10 200 python tools/lane_probe.py > $OUT/lane.txt 2>&1 || exit $?
timeout -k 10 300 python tools/shade_critical.py > $OUT/shade_critical.json 2> $OUT/shade_critical.err || exit $?
tail -1 $OUT/lane.txt; cat $OUT/shade_critical.json
