#!/bin/bash
# r04_index.sh — round 4's one-off GPU session scripts, one function per session, in the order they ran.
# DESIGN.md cites each by name (r04_ab, r04_at, ...); its outputs went to gpurun_out/r04_<name>/ and the kept
# evidence to profiles/r04/.  usage: bash tools/sessions/r04_index.sh <name> [args]   e.g.  ... r04_index.sh ab
# (bodies verbatim apart from the shebang; every session cds to the repo root itself)

r04_a() {
# r04 session A: the launcher-free 2-rank bench test, the default bench line, the one-GPU strong-scaling shard curve (C5, C3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_a; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_a] $(date +%T) pytest gather"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_gather.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gather.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gather.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_a] $(date +%T) bench"
timeout -k 10 300 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
cut -c1-400 $OUT/bench_c3.json
echo "[r04_a] $(date +%T) shard curve c5"
timeout -k 10 300 python tools/shard_curve.py --config c5 > $OUT/shard_c5.json 2> $OUT/shard_c5.err || { tail $OUT/shard_c5.err; exit 1; }
cat $OUT/shard_c5.err | grep '^{'
echo "[r04_a] $(date +%T) shard curve c3"
timeout -k 10 300 python tools/shard_curve.py --config c3 > $OUT/shard_c3.json 2> $OUT/shard_c3.err || { tail $OUT/shard_c3.err; exit 1; }
cat $OUT/shard_c3.err | grep '^{'
}

r04_b() {
# r04 session B: the shading pass's traversal counters (STATS instance), the shaded bench line, the edits tests
# (incremental device ceilings), the C3 full frame (guard counter), the shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_b; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_b] $(date +%T) shade stats"
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
echo "[r04_b] $(date +%T) shade bench"
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
cut -c1-300 $OUT/bench_shade.json
echo "[r04_b] $(date +%T) bench c3"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail $OUT/bench_c3.err; exit 1; }
cut -c1-300 $OUT/bench_c3.json
echo "[r04_b] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_edits.py tests/test_gpu_shade.py "tests/test_gpu_parity.py::test_depth12_full_frame_parity" -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
grep -E "edit \+ sync|passed|failed" $OUT/pytest.log | tail -5; exit $rc
}

r04_c() {
# r04 session C: the fixed / new GPU tests (pick ray highlight pose, the bench's shaded scene over the whole frame,
# C5 last_pos + material, C4 N = 20 at depth 12), the shading pass's traversal counters, the shaded bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_c; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_c] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py "tests/test_gpu_parity.py::test_depth14_4k_sampled_parity" \
    "tests/test_gpu_parity.py::test_ao_depth12_full_frame" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_c] $(date +%T) shade stats"
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
echo "[r04_c] $(date +%T) shade bench"
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
cut -c1-300 $OUT/bench_shade.json
python -c "import json; d=json.load(open('$OUT/bench_shade.json')); print(json.dumps(d['roofline']))"
}

r04_d() {
# r04 session D: shading tests on the working tree, then A/B of the shaded frame: HEAD library (variants/libsvo_base.so)
# against the working tree (the global above-top box and the generalised escape)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_d; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_d] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_d] $(date +%T) A/B"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_d/ab variants/libsvo_base.so default
echo "[r04_d] $(date +%T) shade stats"
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
}

r04_e() {
# r04 session E: shaded frame, ceiling levels 64/256 (working tree) against 16/64 (variants/libsvo_shade1664.so) now that
# rays above the tree's top cross one global box; the parts of the shaded frame (tools/shade_parts.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_e; mkdir -p $OUT; export TMPDIR=/tmp
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_e/ab variants/libsvo_shade1664.so default || exit 1
timeout -k 10 300 python tools/shade_parts.py > $OUT/parts.log 2>&1; rc=$?; cat $OUT/parts.log; exit $rc
}

r04_f() {
# r04 session F: the shading pass walking every ceiling level (max-mipmap, P.ceilq): shading / edits / small-tree tests,
# then A/B against HEAD (libsvo_base) and the global box with 16/64 pairs (libsvo_shade1664); shading counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_f; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_f] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py tests/test_gpu_edits.py tests/test_gpu_small_trees.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "[r04_f] $(date +%T) A/B"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_f/ab variants/libsvo_base.so variants/libsvo_shade1664.so default || exit 1
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
}

r04_g() {
# r04 session G: shading counters with refraction passes, the long tail of bent rays
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
}

r04_h() {
# r04 session H: refractive voxels of a brick passed without lookups: shading tests, A/B against the max-mipmap build
# without it (libsvo_mip) and HEAD (libsvo_base), shading counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_h; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_h] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_h/ab variants/libsvo_base.so variants/libsvo_mip.so default || exit 1
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
}

r04_i() {
# r04 session I: the whole GPU suite on the working tree, then the shaded bench line with its CPU baseline (parity)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_i; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_i] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shade > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_shade.json')); print(d['ms_per_step'], json.dumps(d['roofline'])[:300], d['cpu_baseline'].get('parity_vs_gpu'))"
}

r04_j() {
# r04 session J: split shading (two passes): shading tests, then the shaded frame split (default) against one pass
# (--shade-passes 1) and HEAD's single pass (libsvo_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_j; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_j] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade --shade-passes 1" timeout -k 10 600 bash tools/ab_lib.sh r04_j/ab1 variants/libsvo_base.so default || exit 1
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_j/ab2 default || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --shade --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
cut -c1-120 $OUT/prof/run_kernel_stats.csv | head -8
}

r04_k() {
# r04 session K: dispatch order of the single-pass shading kernel (lake rows sit ~60 % down the frame): top first
# (default), bottom first, 8x8 tiles; and the split shading bottom first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_k; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
for v in "1 0" "1 4" "1 256" "2 4"; do
  set -- $v
  timeout -k 10 120 python bench.py --shade --no-cpu-baseline --steps 30 --shade-passes $1 --cast-flags $2 > $OUT/s$1_f$2_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$OUT/s$1_f$2_$rep.json')); print('passes $1 flags $2', d['ms_per_step'])"
done
done
}

r04_l() {
# r04 session L: the shading instance of the frame's octant casting with the primary's code first (bent rays traced again):
# shading tests, A/B against HEAD (libsvo_base: one reflecting instance for every ray)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_l; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_l] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py tests/test_gpu_bridge.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_l/ab variants/libsvo_base.so default || exit 1
}

r04_m() {
# r04 session M: the shading instance's bounce state (and origin / direction) in LDS instead of spilled registers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_m; mkdir -p $OUT; export TMPDIR=/tmp
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_m/ab variants/libsvo_base.so variants/libsvo_ldsboth.so variants/libsvo_ldsbn.so || exit 1
}

r04_n() {
# r04 session N: bounce state in LDS at 5 (launch bound 8, LDS-limited) vs 6 waves per SIMD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_n/ab variants/libsvo_ldsbn8.so variants/libsvo_w6.so || exit 1
}

r04_o() {
# r04 session O: the working tree (shading bounce state in LDS, 5 waves): the whole GPU suite, shaded bench line with its
# CPU baseline (parity), a rocprofv3 kernel trace of the shaded bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_o; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_o] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shade > $OUT/bench_shade.json 2> $OUT/bench_shade.err || { tail $OUT/bench_shade.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_shade.json')); print(d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'].get('parity_vs_gpu'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shade -o run -- python3 bench.py --shade --steps 10 --warmup 2 --no-cpu-baseline --pipelined-steps 0 > $OUT/bench_prof_shade.json 2> $OUT/prof_shade.err || exit 1
grep k_cast $OUT/prof_shade/run_kernel_stats.csv | cut -c1-160
}

r04_p() {
# r04 session P: the refractive pass continuing into sibling bricks: shading tests, A/B against HEAD, counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_p; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_p] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_p/ab variants/libsvo_base.so default || exit 1
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
}

r04_q() {
# r04 session Q: the refractive pass with the last block's flags cached, without (libsvo_cache) and with (libsvo_sibcache)
# the sibling-brick continuation, against HEAD (libsvo_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_q/ab variants/libsvo_base.so variants/libsvo_cache.so variants/libsvo_sibcache.so || exit 1
}

r04_r() {
# r04 session R: primary casts walking every ceiling level (max-mipmap quads, CEIL 2) against the 16/64 pair (HEAD): C3, C5, C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_r/c3 variants/libsvo_base.so variants/libsvo_quadprim.so || exit 1
REPS=3 BENCH_ARGS="--config c5" timeout -k 10 600 bash tools/ab_lib.sh r04_r/c5 variants/libsvo_base.so variants/libsvo_quadprim.so || exit 1
REPS=3 BENCH_ARGS="--ao 16" timeout -k 10 600 bash tools/ab_lib.sh r04_r/c4 variants/libsvo_base.so variants/libsvo_quadprim.so || exit 1
}

r04_s() {
# r04 session S: ceiling boxes chosen by latest exit among every level the ray is above (f32 estimate): primary casts
# (libsvo_quadlate) against the 16/64 pair (HEAD) and the coarsest level (libsvo_quadprim); the shading pass (libsvo_shadelate)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_s/c3 variants/libsvo_base.so variants/libsvo_quadlate.so || exit 1
REPS=3 BENCH_ARGS="--config c5" timeout -k 10 600 bash tools/ab_lib.sh r04_s/c5 variants/libsvo_base.so variants/libsvo_quadlate.so || exit 1
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_s/shade variants/libsvo_base.so variants/libsvo_shadelate.so || exit 1
}

r04_t() {
# r04 session T: primary casts on the per-level ceiling quads, shallow rays (a_y > K min(a_x, a_z)) taking the coarsest
# block they are above and the others the 16/64 pair's choice: K = 4, 10, against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_t/c3 variants/libsvo_base.so variants/libsvo_hyb4.so variants/libsvo_hyb10.so || exit 1
REPS=3 BENCH_ARGS="--config c5" timeout -k 10 600 bash tools/ab_lib.sh r04_t/c5 variants/libsvo_base.so variants/libsvo_hyb4.so variants/libsvo_hyb10.so || exit 1
}

r04_u() {
# r04 session U: the shading instance without segment-exact crossings (SEG false: integral cameras' rays stay linear, also
# after refraction) against HEAD; its shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_u; mkdir -p $OUT; export TMPDIR=/tmp
SVO_LIB=$PWD/variants/libsvo_shadenoseg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_u/ab variants/libsvo_base.so variants/libsvo_shadenoseg.so || exit 1
}

r04_v() {
# r04 session V: the non-segment shading instance (test + A/B), and the C3 critical path (one-GPU shard curve, N = 1 / 8)
# of the per-level ceiling quads (libsvo_quadprim) against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_v; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/sessions/r04_u.sh || exit 1
for L in base quadprim; do
  SVO_LIB=$PWD/variants/libsvo_$L.so timeout -k 10 300 python tools/shard_curve.py --config c3 --ns 1,8 > $OUT/shard_$L.json 2> $OUT/shard_$L.err || { tail $OUT/shard_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/shard_$L.json')); print('$L', [(r['n'], r['max_us'], round(sum(r['rank_us'])/len(r['rank_us']),1), r['inflight_max_us']) for r in d['curve']])"
done
}

r04_w() {
# r04 session W: PMC passes of the shading pass at the working tree (profiles/pmc_c3_shade.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/pmc.sh r04_w_pmc_shade --shade
}

r04_x() {
# r04 session X: two-phase shading (the frame octant's primary code first, bent rays traced again) on the LDS-bounce
# 5-wave instance, against HEAD; its shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_x; mkdir -p $OUT; export TMPDIR=/tmp
SVO_LIB=$PWD/variants/libsvo_twophase.so timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_x/ab variants/libsvo_base.so variants/libsvo_twophase.so || exit 1
}

r04_y() {
# r04 session Y: shadow rays crossing the scene's column-ceiling boxes (CEIL 1), against HEAD; shading tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_y; mkdir -p $OUT; export TMPDIR=/tmp
SVO_LIB=$PWD/variants/libsvo_shadowceil.so timeout -k 10 600 python -u -m pytest tests/test_gpu_shade.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_y/ab variants/libsvo_base.so variants/libsvo_shadowceil.so || exit 1
}

r04_z() {
# r04 session Z: the gather tests (incl. two frames in flight), C5 strong-mode lines at N = 1 with one and two frames in
# flight, the shaded line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_z; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --frames 1 --inflight $f --no-cpu-baseline > $OUT/c5_strong_if$f.json 2> $OUT/c5_if$f.err || { tail $OUT/c5_if$f.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c5_strong_if$f.json')); print('c5 frames1 inflight $f', d['ms_per_step'], round(d['value']/1e9,2))"
done
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python -c "import json; d=json.load(open('$OUT/shade.json')); print('shade', d['ms_per_step'], d['roofline']['frac'])"
}

r04_aa() {
# r04 session AA: shading with the ceiling quads' coarse levels only after a reflection / refraction (the 16 / 64 choice
# before), against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=5 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_aa/ab variants/libsvo_base.so variants/libsvo_turned.so || exit 1
}

r04_ab() {
# r04 session AB: far-field tile rows (the first K dispatched) crossing 64 / 256-column ceiling boxes instead of 16 / 64
# (experiment library libsvo_far, SVO_FAR_ROWS = K), C3 and C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ab; mkdir -p $OUT; export TMPDIR=/tmp
export SVO_LIB=$PWD/variants/libsvo_far.so
for cfg in c3 c5; do
for rep in 1 2 3; do
for K in 0 8 16 32 64; do
  SVO_FAR_ROWS=$K timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 30 > $OUT/${cfg}_k${K}_$rep.json 2>/dev/null || exit 1
done
done
python3 - $cfg <<'PY'
import json, glob, statistics, sys
cfg = sys.argv[1]
for K in (0, 8, 16, 32, 64):
    ms = [json.load(open(f))['roofline']['avg_launch_ms'] for f in sorted(glob.glob('gpurun_out/r04_ab/%s_k%d_*.json' % (cfg, K)))]
    print(cfg, 'K=%d' % K, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms))
PY
done
}

r04_ac() {
# r04 session AC: the AO instance with its hemisphere table read from the kernel arguments instead of LDS (the LDS then
# allows 8 waves): 7 (71 VGPRs) and 8 waves (64 VGPRs, 4 spilled) against HEAD's 6; C4 at 16 and 20 samples
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--ao 16" timeout -k 10 600 bash tools/ab_lib.sh r04_ac/ao16 variants/libsvo_base.so variants/libsvo_ao7.so variants/libsvo_ao8.so || exit 1
REPS=3 BENCH_ARGS="--ao 20" timeout -k 10 600 bash tools/ab_lib.sh r04_ac/ao20 variants/libsvo_base.so variants/libsvo_ao7.so variants/libsvo_ao8.so || exit 1
}

r04_ad() {
# r04 session AD: the 8-wave AO instance (table from the kernel arguments, no start barrier): the AO / parity tests, then
# C4, C3 and shaded A/B against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ad; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--ao 16" timeout -k 10 600 bash tools/ab_lib.sh r04_ad/c4 variants/libsvo_base.so default || exit 1
REPS=4 timeout -k 10 600 bash tools/ab_lib.sh r04_ad/c3 variants/libsvo_base.so default || exit 1
REPS=3 BENCH_ARGS="--shade" timeout -k 10 600 bash tools/ab_lib.sh r04_ad/shade variants/libsvo_base.so default || exit 1
}

r04_ae() {
# r04 session AE: the wire decode on 32-bit divisions: wire / gather tests, the exchange parts, the 1-rank exchange lines
# against HEAD (libsvo_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ae; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "wire or exchange or multi_frame or sharding" tests/test_gpu_bench_gather.py tests/test_gpu_bridge.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in base default; do
  if [ $L = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/variants/libsvo_$L.so; fi
  timeout -k 10 300 python tools/xchg_parts.py > $OUT/parts_$L.log 2>&1 || { tail $OUT/parts_$L.log; exit 1; }
  echo "== $L"; cat $OUT/parts_$L.log | grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl"
done
unset SVO_LIB
REPS=4 BENCH_ARGS="--force-exchange --no-cpu-baseline" timeout -k 10 600 bash tools/ab_lib.sh r04_ae/x3 variants/libsvo_base.so default || exit 1
}

r04_af() {
# r04 session AF: the 1-rank exchange's step cost with the cast streams at high priority against normal (C3, C5 --frames 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_af; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3 4; do
for p in 0 1; do
  timeout -k 10 120 python bench.py --force-exchange --no-cpu-baseline --steps 30 --cast-priority $p > $OUT/c3_p${p}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py --config c5 --frames 1 --force-exchange --no-cpu-baseline --steps 20 --cast-priority $p > $OUT/c5_p${p}_$rep.json 2>/dev/null || exit 1
done
done
python3 - <<'PY'
import json, glob, statistics
for c in ('c3', 'c5'):
    for p in (0, 1):
        ms = [json.loads([l for l in open(f) if l.startswith('{')][-1])['ms_per_step'] for f in sorted(glob.glob('gpurun_out/r04_af/%s_p%d_*.json' % (c, p)))]
        print(c, 'priority', p, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms))
PY
}

r04_ag() {
# r04 session AG: the parts of the shaded frame at the round's build (tools/shade_parts.py), and its counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ag; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_parts.py > $OUT/parts.log 2>&1 || { tail $OUT/parts.log; exit 1; }
grep -v amdgpu.ids $OUT/parts.log
timeout -k 10 300 python tools/shade_stats.py > $OUT/shade_stats.json 2> $OUT/shade_stats.err || { tail $OUT/shade_stats.err; exit 1; }
cat $OUT/shade_stats.json
}

r04_ah() {
# r04 session AH: occupancy sensitivity of the primary instance: 5 and 6 waves per SIMD against 8 (C3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=3 timeout -k 10 600 bash tools/ab_lib.sh r04_ah/c3 variants/libsvo_base.so variants/libsvo_prim5.so variants/libsvo_prim6.so || exit 1
}

r04_ai() {
# r04 session AI: wavefront footprint per config — 16x4 (default), 8x8 (flag 256), 32x2 (flag 512) at C3, C5, C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ai; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
for cfg in "c3" "c5" "c3 --ao 16"; do
for fl in 0 256 512; do
  tag=$(echo "$cfg" | tr -d ' -')
  timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 30 --cast-flags $fl > $OUT/${tag}_f${fl}_$rep.json 2>/dev/null || exit 1
done
done
done
python3 - <<'PY'
import json, glob, statistics
for tag in ('c3', 'c5', 'c3ao16'):
    for fl in (0, 256, 512):
        ms = [json.load(open(f))['roofline']['avg_launch_ms'] for f in sorted(glob.glob('gpurun_out/r04_ai/%s_f%d_*.json' % (tag, fl)))]
        print(tag, 'flags', fl, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms))
PY
}

r04_aj() {
# r04 session AJ: PMC passes of C4 (the 8-wave AO instance) and C5 at the round's build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/pmc.sh r04_aj/pmc_c4 --ao 16 > gpurun_out/r04_aj_c4.log 2>&1 || { tail gpurun_out/r04_aj_c4.log; exit 1; }
tail -4 gpurun_out/r04_aj_c4.log
bash tools/pmc.sh r04_aj/pmc_c5 --config c5 > gpurun_out/r04_aj_c5.log 2>&1 || { tail gpurun_out/r04_aj_c5.log; exit 1; }
tail -4 gpurun_out/r04_aj_c5.log
}

r04_ak() {
# r04 session AK: gloo rehearsals of more ranks on one GPU — weak C3 at N = 4 and 6, strong C5 (one 4K frame) at N = 4 with
# two frames in flight; every displayed frame verified against a one-GPU cast
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ak; mkdir -p $OUT; export TMPDIR=/tmp
d() { local name=$1 n=$2 port=$3; shift 3; echo "[ak] $(date +%T) $name"; timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --dist-backend gloo "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$name.err; exit $rc; }; grep '^{' $OUT/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['n_gpus'], d['scaling'], round(d['value']/1e6,1), 'M rays/s', 'verified', d.get('gather_verified'))"; }
d g4_weak 4 29651 --steps 4 --warmup 1 --verify
d g6_weak 6 29652 --steps 3 --warmup 1 --verify
d g4_c5_strong_if2 4 29653 --config c5 --frames 1 --inflight 2 --steps 4 --warmup 1 --verify
# the 1-rank exchange's kernels (C3): the fused cast and the decode, from a kernel trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_x1 -o run -- python3 bench.py --force-exchange --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_x1.json 2> $OUT/prof_x1.err || exit 1
cut -c1-150 $OUT/prof_x1/run_kernel_stats.csv | head -6
}

r04_al() {
# r04 session AL: three buffer sets with an exchange: the 1-rank RCCL exchange lines (C3, C5 --frames 1, C4) against two
# (git stash of bench.py is not available on the box: --nbuf-exchange is not an option, so HEAD's bench.py is compared via
# its copy bench_nbuf2.py), the gather tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_al; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for b in bench bench_nbuf2; do
  timeout -k 10 120 python $b.py --force-exchange --verify --no-cpu-baseline --steps 30 > $OUT/c3_${b}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python $b.py --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline --steps 20 > $OUT/c5_${b}_$rep.json 2>/dev/null || exit 1
done
done
python3 - <<'PY'
import json, glob, statistics
for c in ('c3', 'c5'):
    for b in ('bench', 'bench_nbuf2'):
        ds = [json.loads([l for l in open(f) if l.startswith('{')][-1]) for f in sorted(glob.glob('gpurun_out/r04_al/%s_%s_*.json' % (c, b)))]
        ms = [d['ms_per_step'] for d in ds]
        print(c, b, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms), 'verified', all(d.get('gather_verified') for d in ds))
PY
}

r04_am() {
# r04 session AM: is the 1-rank exchange step host-bound? (tools/xchg_host.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_am; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/xchg_host.py > $OUT/host.log 2>&1; rc=$?; grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids" $OUT/host.log; exit $rc
}

r04_an() {
# r04 session AN: bench.py timing the region with one event pair on the cast stream(s) also with an exchange / two
# frames in flight (per-launch timing events serialised the streams): forced 1-rank exchange lines against HEAD's
# bench.py (bench_old.py), the gather tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_an; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_gather.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for b in bench bench_old; do
  timeout -k 10 120 python $b.py --force-exchange --verify --no-cpu-baseline --steps 30 > $OUT/c3_${b}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python $b.py --config c5 --frames 1 --force-exchange --verify --no-cpu-baseline --steps 20 > $OUT/c5_${b}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python $b.py --config c5 --frames 1 --inflight 2 --no-cpu-baseline --steps 20 > $OUT/c5if_${b}_$rep.json 2>/dev/null || exit 1
done
done
python3 - <<'PY'
import json, glob, statistics
for c in ('c3', 'c5', 'c5if'):
    for b in ('bench', 'bench_old'):
        ds = [json.loads([l for l in open(f) if l.startswith('{')][-1]) for f in sorted(glob.glob('gpurun_out/r04_an/%s_%s_[0-9].json' % (c, b)))]
        ms = [d['ms_per_step'] for d in ds]
        print(c, b, 'median %.4f' % statistics.median(ms), ' '.join('%.4f' % m for m in ms), 'verified', [d.get('gather_verified') for d in ds],
              'avg_launch', ds[0]['roofline']['avg_launch_ms'])
PY
}

r04_ao() {
# r04 session AO: the exchange's decode in one-wave blocks (it runs beside the next cast): forced 1-rank exchange lines
# against HEAD (libsvo_base); the wire / gather tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ao; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "wire or exchange" tests/test_gpu_bench_gather.py tests/test_gpu_bridge.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--force-exchange --verify" timeout -k 10 600 bash tools/ab_lib.sh r04_ao/c3 variants/libsvo_base.so default || exit 1
REPS=3 BENCH_ARGS="--config c5 --frames 1 --force-exchange --verify" timeout -k 10 600 bash tools/ab_lib.sh r04_ao/c5 variants/libsvo_base.so default || exit 1
}

r04_ap() {
# r04 session AP: the exchange's decode in 512- and 1024-thread blocks (held back to the next cast's tail) against 256
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--force-exchange" timeout -k 10 600 bash tools/ab_lib.sh r04_ap/c3 variants/libsvo_base.so variants/libsvo_sc512.so variants/libsvo_sc1024.so || exit 1
}

r04_aq() {
# r04 session AQ: the 1024-thread decode: wire / exchange / gather / bridge tests, the forced 1-rank exchange lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_aq; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "wire or exchange or multi_frame or sharding" tests/test_gpu_bench_gather.py tests/test_gpu_bridge.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in "xchg1 --force-exchange --verify" "xchg1_ao --force-exchange --verify --ao 16" "c5_xchg1 --config c5 --frames 1 --force-exchange --verify"; do
  set -- $c; name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  grep '^{' $OUT/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], round(d['value']/1e9,2), d.get('gather_verified'))"
done
}

r04_ar() {
# r04 session AR: the builders' ceiling tables (host vs GPU terrain builders), the build tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ar; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_build.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; exit $rc
}

r04_as() {
# r04 session AS: the shaded frame's per-block timeline (tools/shade_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_as; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_timeline.py gpurun_out/r04_as/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
cat $OUT/timeline.json
}

r04_at() {
# r04 session AT: frame schedules (longest block first from the last frame): parity, then A/B against the default order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_at; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
REPS=3 BENCH_ARGS="--shade" bash tools/ab_flags.sh r04_at/shade 0 65536 || exit 1
REPS=3 bash tools/ab_flags.sh r04_at/c3 0 65536 || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_flags.sh r04_at/c5 0 65536 || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_flags.sh r04_at/c4 0 65536 || exit 1
timeout -k 10 300 python tools/shade_timeline.py $OUT/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || exit 1
cut -c1-600 $OUT/timeline.json
}

r04_au() {
# r04 session AU: shading-only frame schedules: schedule + shading GPU tests, shaded bench line, its kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_au; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_shade.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['config']['dispatch_order'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; cut -c1-200 $OUT/kernel_stats_shade.csv | head -8
}

r04_av() {
# r04 session AV: block timelines after the shading schedule (primary: default order) (tools/shade_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_av; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_timeline.py gpurun_out/r04_av/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
cat $OUT/timeline.json
}

r04_aw() {
# r04 session AW: block timelines with the shading schedule (primary in its default order); shading waves per SIMD
# under the schedule (4 / 5 / 6, variants built by tools/build_variant.py --patch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_aw; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/shade_timeline.py $OUT/stamps.npz > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
cut -c1-300 $OUT/timeline.json
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r04_aw/shade default variants/libsvo_shade_w4.so variants/libsvo_shade_w6.so
}

r04_ax() {
# r04 session AX: the sort kernel with batched loads and logarithmic buckets: schedule tests, shaded bench line, its
# kernel trace (k_sched_order's duration), and the schedule under camera motion (tools/shade_motion.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ax; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; grep -E "k_cast|k_sched" $OUT/kernel_stats_shade.csv | cut -d, -f2-4 
timeout -k 10 400 python tools/shade_motion.py 40 > $OUT/motion.log 2> $OUT/motion.err || { tail $OUT/motion.err; exit 1; }
cat $OUT/motion.log
}

r04_ay() {
# r04 session AY: one load round in the sort kernel; the schedule gated on camera motion: schedule tests, shaded bench line, its
# kernel trace (k_sched_order's duration), and the schedule under camera motion (tools/shade_motion.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ay; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; grep -E "k_cast|k_sched" $OUT/kernel_stats_shade.csv | cut -d, -f2-4 
timeout -k 10 400 python tools/shade_motion.py 40 > $OUT/motion.log 2> $OUT/motion.err || { tail $OUT/motion.err; exit 1; }
cat $OUT/motion.log
}

r04_az() {
# r04 session AZ: the schedule by groups of 4 blocks (a quarter of the sort): schedule tests, shaded bench line, its
# kernel trace (k_sched_order's duration), and the schedule under camera motion (tools/shade_motion.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_az; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; grep -E "k_cast|k_sched" $OUT/kernel_stats_shade.csv | cut -d, -f2-4 
timeout -k 10 400 python tools/shade_motion.py 40 > $OUT/motion.log 2> $OUT/motion.err || { tail $OUT/motion.err; exit 1; }
cat $OUT/motion.log
}

r04_ba() {
# r04 session BA: no sort after a frame whose camera moved too far: schedule tests, shaded bench line, its
# kernel trace (k_sched_order's duration), and the schedule under camera motion (tools/shade_motion.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_ba; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --shade --steps 50 --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('$OUT/shade.json') if l.startswith('{')][-1]); print('shade', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o shade -- python3 bench.py --shade --steps 50 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_shade.csv; grep -E "k_cast|k_sched" $OUT/kernel_stats_shade.csv | cut -d, -f2-4 
timeout -k 10 400 python tools/shade_motion.py 40 > $OUT/motion.log 2> $OUT/motion.err || { tail $OUT/motion.err; exit 1; }
cat $OUT/motion.log
}

r04_bb() {
# r04 session BB: primary casts under the grouped, camera-gated frame schedule (a variant that attaches it to primary
# and AO launches too) against the shipped default order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04_bb; export TMPDIR=/tmp
REPS=3 bash tools/ab_lib.sh r04_bb/c3 default variants/libsvo_prim_sched.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r04_bb/c5 default variants/libsvo_prim_sched.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r04_bb/c4 default variants/libsvo_prim_sched.so || exit 1
}

r04_bc() {
# r04 session BC: host time of edit + update + sync (tools/edit_sync_timing.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_bc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/edit_sync_timing.py > $OUT/edit_sync.json 2> $OUT/edit_sync.err || { tail $OUT/edit_sync.err; exit 1; }
cat $OUT/edit_sync.json
}

r04_bd() {
# r04 session BD: the shading schedule by groups of 8 blocks (variant) against groups of 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04_bd; export TMPDIR=/tmp
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r04_bd/shade default variants/libsvo_sched_g8.so || exit 1
}

r04_be() {
# r04 session BE: PMC passes of the shading instance with the frame schedule (warmup 3: the timed launches scheduled)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/pmc.sh r04_be/pmc_shade --shade --warmup 3 > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04_be/pmc_shade/pmc_summary.json')); print({k: d[k] for k in ('hbm_bytes_per_launch', 'l2_hit_rate', 'valu_per_wave', 'salu_per_wave', 'bench_avg_launch_ms') if k in d})"
}

r04_bf() {
# r04 session BF: the schedule tests with the camera-motion gate test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_bf; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; exit $rc
}

r04_bg() {
# r04 session BG: the whole GPU suite and smoke at the round's last commit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_bg; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cut -c1-200 $OUT/bench.json
}

r04_bh() {
# r04 session BH: C5's block timeline (bench.py --stats with SVO_STAMPS) — is the 4K launch bound by its longest waves?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04_bh; mkdir -p $OUT; export TMPDIR=/tmp
SVO_STAMPS=$OUT/stamps_c5.npy timeout -k 10 300 python bench.py --config c5 --stats --steps 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5_stats.err || { tail $OUT/c5_stats.err; exit 1; }
tail -25 $OUT/c5_stats.err
}

r04_final() {
# r04 final evidence: the GPU suite, then tools/evidence.sh (every config's bench line with its CPU baseline, the 1-rank
# RCCL exchange, gloo rehearsals, rocprofv3 kernel traces), then the C3 PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${R04_FINAL_TAG:-r04_final}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r04_final] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/evidence.sh ${R04_FINAL_TAG:-r04_final}/ev || exit $?
bash tools/pmc.sh ${R04_FINAL_TAG:-r04_final}/pmc_c3 > $OUT/pmc_c3.log 2>&1 || { tail $OUT/pmc_c3.log; exit 1; }
tail -3 $OUT/pmc_c3.log
}

name=${1:?usage: r04_index.sh <session name: a b c d e f g h i j k l m n o p q r s t u v w x y z aa ab ac ad ae af ag ah ai aj ak al am an ao ap aq ar as at au av aw ax ay az ba bb bc bd be bf bg bh final>}
shift
case " a b c d e f g h i j k l m n o p q r s t u v w x y z aa ab ac ad ae af ag ah ai aj ak al am an ao ap aq ar as at au av aw ax ay az ba bb bc bd be bf bg bh final " in *" $name "*) "r04_$name" "$@" ;; *) echo "no session r04_$name" >&2; exit 2 ;; esac
