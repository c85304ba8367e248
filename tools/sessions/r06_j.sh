# r06 j: strong-scaling shard curves of the final build (C5 and C3, N = 1, 2, 4, 8, one launch at a time and two in
# flight; VERDICT r05 item 1's C5 N = 8 target)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06_j; mkdir -p $OUT
sha256sum raytracing_test_amd/libsvo_rt.so | tee $OUT/lib_sha256.txt
timeout -k 10 300 python -u tools/shard_curve.py --config c5 > $OUT/shard_curve_c5.json 2> $OUT/shard_c5.err || { tail $OUT/shard_c5.err; exit 1; }
timeout -k 10 300 python -u tools/shard_curve.py --config c3 > $OUT/shard_curve_c3.json 2> $OUT/shard_c3.err || { tail $OUT/shard_c3.err; exit 1; }
cat $OUT/shard_curve_c5.json $OUT/shard_curve_c3.json
# the shaded frame's per-block timeline in its scheduled order: do the blocks that end last start late?
timeout -k 10 300 python -u tools/shade_timeline.py $OUT/shade_timeline.npz > $OUT/shade_timeline.json 2> $OUT/shade_timeline.err || { tail $OUT/shade_timeline.err; exit 1; }
cat $OUT/shade_timeline.json
