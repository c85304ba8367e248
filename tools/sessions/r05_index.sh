#!/bin/bash
# r05_index.sh — round 5's one-off GPU session scripts, one function per session, in the order they ran.
# DESIGN.md cites each by name (r05_l, r05_v, ..., pmc, final); its outputs went to gpurun_out/r05_<name>*/ and the kept
# evidence to profiles/r05/ and profiles/r05_*.  usage: bash tools/sessions/r05_index.sh <name> [args]   e.g.  ... r05_index.sh final
# (bodies verbatim apart from the shebang; every session cds to the repo root itself)

r05_a() {
# r05_a: baseline of the round's starting library on this box: C3 bench x3, shaded x2, C5 x1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_a; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $OUT/c3_$i.json 2> $OUT/c3_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --shade > $OUT/shade_$i.json 2> $OUT/shade_$i.err || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --config c5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' $OUT/*.json
}

r05_b() {
# r05_b: the bridge (main.cpp-shaped TU) and the N > 1 C-ABI exchange through the RCCL stand-in, on one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bridge.py tests/test_gpu_bench_gather.py > $OUT/pytest.log 2>&1
rc=$?; tail -30 $OUT/pytest.log; exit $rc
}

r05_c() {
# r05_c: per-block stamps + per-ray work of one C3 frame (STATS / TIMELINE instances), and the top-rows probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_c; mkdir -p $OUT
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/bench.json 2> $OUT/stats.txt || exit 1
timeout -k 10 300 python tools/tail_probe.py > $OUT/tail_probe.txt 2>&1 || exit 1
cat $OUT/stats.txt $OUT/tail_probe.txt | tail -30
}

r05_d() {
# r05_d: the whole GPU suite after the ADVICE r04 fixes (shadow-ray ceilings, escape vs look-at, schedule lock, syncs),
# then C3 and shaded benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_d; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $OUT/c3_$i.json 2> $OUT/c3_$i.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --shade > $OUT/shade_$i.json 2> $OUT/shade_$i.err || exit 1
done
grep -h -o '"ms_per_step": [0-9.]*' $OUT/*.json
exit $rc
}

r05_e() {
# r05_e: critical-path probe — far-field waves with fewer rays per wave (tools/lane_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_e; mkdir -p $OUT
timeout -k 10 600 python tools/lane_probe.py > $OUT/lane_probe.txt 2> $OUT/lane_probe.err; rc=$?
tail -1 $OUT/lane_probe.txt; tail -3 $OUT/lane_probe.err; exit $rc
}

r05_f() {
# r05_f: A/B of the column-ceiling granularity: 4-column finest level (SVO_CEIL_K0 1; primary pairs 4/16 or 4/64)
# against the shipped 16/64 — C3, C5, shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=3 bash tools/ab_lib.sh r05_f_c3 default variants/libsvo_k01.so variants/libsvo_k01p02.so || exit 1
REPS=2 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_f_c5 default variants/libsvo_k01.so variants/libsvo_k01p02.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_f_sh default variants/libsvo_k01.so variants/libsvo_k01p02.so || exit 1
}

r05_g() {
# r05_g: column-ceiling granularity, second A/B: primary pairs 4/64 (k01p02), 4/256 (k1p03), shadow pairs 4/64 (k1p02s02),
# 1-column finest level (k0p03: 1/64, k0p13: 4/64) — C3, C5, shaded C3, C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
V="default variants/libsvo_k01p02.so variants/libsvo_k1p03.so variants/libsvo_k1p02s02.so variants/libsvo_k0p03.so variants/libsvo_k0p13.so"
REPS=3 bash tools/ab_lib.sh r05_g_c3 $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_g_sh $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_g_ao $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_g_c5 default variants/libsvo_k01p02.so variants/libsvo_k1p03.so || exit 1
}

r05_h() {
# r05_h: column-ceiling layouts with the pair table's partner level configurable (SVO_CEIL_PAIR_STEP): finest level
# 4 or 16 columns (SVO_CEIL_K0 1 / 2), second level 2 or 3 levels up — parity of each variant (the whole C3 frame, the
# edits' tables), then A/B C3, C5, C4, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_h; mkdir -p $OUT
for v in k1s2 k1s3 k2s2 k2s3; do
  SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_edits.py tests/test_gpu_small_trees.py -k "depth12 or edits or small or ceiling or frame" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ge 124 ] && exit $rc
done
V="default variants/libsvo_k1s2.so variants/libsvo_k1s3.so variants/libsvo_k2s2.so variants/libsvo_k2s3.so"
REPS=3 bash tools/ab_lib.sh r05_h_c3 $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_h_sh $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_h_ao $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_h_c5 $V || exit 1
}

r05_i() {
# r05_i: clock probe — far-field waves alone vs inside the whole frame: duration, shader cycles, clock
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_i; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_clock.so timeout -k 10 300 python tools/clock_probe.py > $OUT/clock_probe.txt 2> $OUT/clock_probe.err; rc=$?
cat $OUT/clock_probe.txt; tail -3 $OUT/clock_probe.err; exit $rc
}

r05_j() {
# r05_j: the top tile rows alone (tools/tail_probe.py) on each ceiling layout: does a finer / coarser layout shorten the
# far-field critical path although it slows the whole frame?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_j; mkdir -p $OUT
for v in default k1s2 k2s2 k1s3; do
  if [ $v = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/variants/libsvo_$v.so; fi
  timeout -k 10 200 python tools/tail_probe.py --reps 10 > $OUT/tail_$v.txt 2>/dev/null || exit 1
  echo "$v $(tail -1 $OUT/tail_$v.txt)"
done
}

r05_k() {
# r05_k: where the shaded frame's time goes now: plain cast, shaded with / without shadow rays, without water
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_k; mkdir -p $OUT
timeout -k 10 300 python tools/shade_parts.py > $OUT/shade_parts.txt 2> $OUT/shade_parts.err; rc=$?
cat $OUT/shade_parts.txt; exit $rc
}

r05_l() {
# r05_l: the column-ceiling march (ceil_march) — parity (parity, configs, small trees, edits, large, AO), then A/B against
# the round's previous commit (variants/libsvo_base.so): C3, C4, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_edits.py tests/test_gpu_large.py tests/test_gpu_build.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_l_c3 variants/libsvo_base.so default || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_l_ao variants/libsvo_base.so default || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_l_c5 variants/libsvo_base.so default || exit 1
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/stats.json 2> $OUT/stats.txt
grep "stats per ray" $OUT/stats.txt | head -2
}

r05_m() {
# r05_m: the march inside the loop too (every ceiling move of a descending ray marches on) vs the pre-loop march only:
# parity of the in-loop build, then A/B C3, C4, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_m; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_inloop.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_edits.py tests/test_gpu_large.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_m_c3 variants/libsvo_pre.so variants/libsvo_inloop.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_m_ao variants/libsvo_pre.so variants/libsvo_inloop.so || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_m_c5 variants/libsvo_pre.so variants/libsvo_inloop.so || exit 1
}

r05_n() {
# r05_n: 1/absDelta recomputed per use (Ray.ia dropped: no spill with the march) vs the march commit — parity, A/B C3, C4,
# C5, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_n; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_noia.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_shade.py > $OUT/pytest.log 2>&1
SVO_LIB=$PWD/variants/libsvo_shmarch.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest_sh.log 2>&1; rc2=$?; echo "shmarch pytest rc=$rc2: $(tail -1 $OUT/pytest_sh.log)"
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_n_c3 variants/libsvo_pre.so variants/libsvo_noia.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_n_ao variants/libsvo_pre.so variants/libsvo_noia.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_n_sh variants/libsvo_pre.so variants/libsvo_noia.so variants/libsvo_shmarch.so || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_n_c5 variants/libsvo_pre.so variants/libsvo_noia.so || exit 1
}

r05_o() {
# r05_o: the march in the shading trace too (stored 1/absDelta kept) — the whole GPU suite, then A/B shaded / C3 vs the
# march commit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_o; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_o_sh variants/libsvo_pre.so default || exit 1
REPS=3 bash tools/ab_lib.sh r05_o_c3 variants/libsvo_pre.so default || exit 1
}

r05_p() {
# r05_p: after the march — the top tile rows alone (critical path) and the per-block timeline / per-ray work of C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_p; mkdir -p $OUT
timeout -k 10 200 python tools/tail_probe.py --reps 10 > $OUT/tail.txt 2>/dev/null || exit 1
tail -1 $OUT/tail.txt
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/stats.json 2> $OUT/stats.txt || exit 1
grep "stats per ray\|timeline" $OUT/stats.txt
}

r05_q() {
# r05_q: the slim march (no entry-event double) and 1/absDelta set after the march (no spill) vs HEAD — parity of the
# product build, A/B C3, C4, C5, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_q; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_shade.py tests/test_gpu_edits.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
V="variants/libsvo_pre2.so variants/libsvo_slim.so variants/libsvo_slimrcp.so"
REPS=3 bash tools/ab_lib.sh r05_q_c3 $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_q_ao $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_q_sh $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_q_c5 $V || exit 1
}

r05_r() {
# r05_r: the march with two blocks of ceiling prefetch (and 1/absDelta set after it) vs HEAD — parity, A/B C3, C4, C5, shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_r; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_d2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_small_trees.py tests/test_gpu_shade.py tests/test_gpu_edits.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
V="variants/libsvo_pre2.so variants/libsvo_d2.so"
REPS=3 bash tools/ab_lib.sh r05_r_c3 $V || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_r_ao $V || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_r_sh $V || exit 1
REPS=1 BENCH_ARGS="--config c5 --steps 10" bash tools/ab_lib.sh r05_r_c5 $V || exit 1
}

r05_s() {
# r05_s: shadow rays climb on through the blocks they stay above (ceil_climb) — shading parity, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_s; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_climb.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_s_sh variants/libsvo_pre2.so variants/libsvo_climb.so || exit 1
}

r05_t() {
# r05_t: REFLECT sign flags re-derived only after a bounce (flags); + shading launches without hit records keep no
# crossing value (norec) — shading parity, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_t; mkdir -p $OUT
for v in flags norec; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest_$v.log 2>&1
rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_$v.log | head -20; exit $rc; }
done
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_t_sh variants/libsvo_pre2.so variants/libsvo_flags.so variants/libsvo_norec.so || exit 1
}

r05_u() {
# r05_u: shading launches without hit records keep no crossing value (norec2, on HEAD); diagnostic: the shading trace
# without the reflection / refraction machinery (norefl: wrong images, timing only) — parity of norec2, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_u; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_norec2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_u_sh variants/libsvo_pre2.so variants/libsvo_norec2.so variants/libsvo_norefl.so || exit 1
}

r05_v() {
# r05_v: shading rays trace straight to their first hit, and only mirrors / refractive blocks with budget left resume
# in the bouncing trace (split) — shading parity, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_v; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_split.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_v_sh variants/libsvo_norec2.so variants/libsvo_split.so || exit 1
}

r05_w() {
# r05_w: the straight trace of shading rays on the camera's step octant (cam; shadow rays then take generic sign flags),
# the same at 6 waves per SIMD (cam6) — shading parity, A/B shaded C3 against split (r05_v) and HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_w; mkdir -p $OUT
for v in cam cam6; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest_$v.log 2>&1
rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_$v.log | head -20; exit $rc; }
done
REPS=3 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_w_sh variants/libsvo_norec2.so variants/libsvo_split.so variants/libsvo_cam.so variants/libsvo_cam6.so || exit 1
}

r05_x() {
# r05_x: the straight shading trace on the launch's two ceiling levels (cam1: CEIL 1, as primary casts) instead of
# the walk over every level (cam6: CEIL 2) — shading parity, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_x; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_cam1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_x_sh variants/libsvo_cam6.so variants/libsvo_cam1.so || exit 1
}

r05_y() {
# r05_y: the product build with the split shading trace (camera octant, CEIL 1, 6 waves): full GPU suite, shaded and
# plain C3 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/shade.json 2>$OUT/shade.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c3.json 2>$OUT/c3.err || exit 1
python3 -c "
import json
for n in ('shade','c3'):
    d=json.loads([l for l in open('$OUT/%s.json'%n) if l.startswith('{')][-1]); r=d.get('roofline') or {}
    print(n, d['ms_per_step'], r.get('avg_launch_ms'))"
}

r05_z() {
# r05_z: the ceiling march takes the parent block's ceiling (no load) for the blocks inside a parent the ray stays above
# (pmarch) — full GPU suite on it, A/B C3 / C4 / C5 / shaded against the HEAD build (h9f)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_z; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_pmarch.so timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 bash tools/ab_lib.sh r05_z_c3 variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_z_ao variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r05_z_c5 variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_z_sh variants/libsvo_h9f.so variants/libsvo_pmarch.so || exit 1
}

r05_aa() {
# r05_aa: where the C3 critical path stands after the ceiling march: per-wave work of the longest waves (STATS build
# stamps + per-ray work), the shard curve (N = 1..8, one launch at a time and in flight)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_aa; mkdir -p $OUT
SVO_STAMPS=$OUT/stamps.npy SVO_RAY_WORK=$OUT/work.npy timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --stats > $OUT/bench.json 2> $OUT/bench.err || exit 1
python tools/wave_work.py $OUT/stamps.npy $OUT/work.npy > $OUT/wave_work.txt 2>&1; echo "wave_work rc=$?"
timeout -k 10 300 python tools/shard_curve.py --config c3 > $OUT/shard_c3.json 2> $OUT/shard_c3.err || exit 1
timeout -k 10 300 python tools/shard_curve.py --config c5 > $OUT/shard_c5.json 2> $OUT/shard_c5.err || exit 1
head -30 $OUT/wave_work.txt
python3 -c "
import json
for c in ('c3','c5'):
    d=json.loads([l for l in open('$OUT/shard_%s.json'%c) if l.startswith('{')][-1])
    for e in d['curve']: print(c, e['n'], e['max_us'], e['ideal_us'], e.get('inflight_max_us'), e['rank_us'])"
}

r05_pmc() {
# r05_pmc: PMC passes of every bench config on the product build (commit 9f8e7ae's library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
sha256sum raytracing_test_amd/libsvo_rt.so
bash tools/pmc_all.sh r05_pmc || exit $?
}

r05_final() {
# r05 final evidence: the GPU suite, smoke, then tools/evidence.sh (every config's bench line with its CPU baseline, the
# 1-rank RCCL exchange, gloo rehearsals, the C-ABI exchange at N = 2 / 3 over the test-only stand-in, rocprofv3 kernel
# traces) on the library whose PMC passes are in profiles/pmc_*.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${R05_FINAL_TAG:-r05_final}; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
echo "[r05_final] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/evidence.sh ${R05_FINAL_TAG:-r05_final}/ev || exit $?
}

r05_ab() {
# r05_ab: the record index taken again after the trace (rec: primary instances without spills) and the primary
# instances at 7 waves (w7, 66 VGPRs, no spills) against the HEAD build (h9f) — full GPU suite on rec, A/B C3 / C4 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ab; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_rec.so timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 bash tools/ab_lib.sh r05_ab_c3 variants/libsvo_h9f.so variants/libsvo_rec.so variants/libsvo_w7.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_ab_ao variants/libsvo_h9f.so variants/libsvo_rec.so variants/libsvo_w7.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r05_ab_c5 variants/libsvo_h9f.so variants/libsvo_rec.so variants/libsvo_w7.so || exit 1
}

r05_ac() {
# r05_ac: shadow rays with wave-uniform sign flags in scalar registers (uni) — shading parity, A/B shaded C3 vs h9f
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ac; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_uni.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_ac_sh variants/libsvo_h9f.so variants/libsvo_uni.so || exit 1
}

r05_ad() {
# r05_ad: where the shaded frame's time goes on the split build (tools/shade_parts.py), and the frame schedule on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ad; mkdir -p $OUT
timeout -k 10 300 python tools/shade_parts.py > $OUT/shade_parts.txt 2>&1 || { tail $OUT/shade_parts.txt; exit 1; }
cat $OUT/shade_parts.txt
for rep in 1 2 3; do
timeout -k 10 120 python bench.py --shade --no-cpu-baseline --steps 30 > $OUT/sched_on_$rep.json 2>/dev/null || exit 1
timeout -k 10 120 python bench.py --shade --no-cpu-baseline --steps 30 --cast-flags 65536 > $OUT/sched_off_$rep.json 2>/dev/null || exit 1
done
python3 -c "
import json
for m in ('on','off'):
    print('schedule', m, [json.loads([l for l in open('$OUT/sched_%s_%d.json'%(m,r)) if l.startswith('{')][-1])['ms_per_step'] for r in (1,2,3)])"
}

r05_ae() {
# r05_ae: the shading pass's straight trace without segment bounds when every origin is exact (seg0: need_seg) — shading
# parity, A/B shaded C3 against the final build (h18 = 18957fa5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ae; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_seg0.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_ae_sh variants/libsvo_h18.so variants/libsvo_seg0.so || exit 1
}

r05_final3() {
# r05_final3: the final build (the straight shading trace without segment bounds for exact origins): the GPU suite,
# smoke, every config's PMC passes (copied into this box's profiles/ so the bench lines read them), then tools/evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_final3; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
echo "[r05_final3] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_all.sh r05_pmc3 || exit $?
for k in c3 c3f c3_ao16 c5 c3_shade c2; do cp gpurun_out/r05_pmc3_$k/pmc_summary.json profiles/pmc_$k.json || exit 1; done
bash tools/evidence.sh r05_final3/ev || exit $?
}

r05_af() {
# r05_af: DIAGNOSTIC (levels-6 trees only: a 5-level LDS path) — the shading kernel at 7 waves (72 VGPRs, the bent flag
# packed into the reflection count, LDS 5.6 KB per block) against the final build (de28): shaded C3 timing only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_af_sh variants/libsvo_de28.so variants/libsvo_s7.so || exit 1
}

r05_ag() {
# r05_ag: the shading kernel at 7 waves for real (the launch's own LDS path depth, the bent flag packed: s7b = the
# product build) — the full GPU suite on it, A/B shaded C3 / C3 / C4 / C5 against de28 (the previous final build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ag; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_ag_sh variants/libsvo_de28.so variants/libsvo_s7b.so || exit 1
REPS=3 bash tools/ab_lib.sh r05_ag_c3 variants/libsvo_de28.so variants/libsvo_s7b.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_ag_ao variants/libsvo_de28.so variants/libsvo_s7b.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r05_ag_c5 variants/libsvo_de28.so variants/libsvo_s7b.so || exit 1
}

r05_final4() {
# r05_final4: the final build (the shading instances at 7 waves): the GPU suite,
# smoke, every config's PMC passes (copied into this box's profiles/ so the bench lines read them), then tools/evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_final4; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
echo "[r05_final4] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_all.sh r05_pmc4 || exit $?
for k in c3 c3f c3_ao16 c5 c3_shade c2; do cp gpurun_out/r05_pmc4_$k/pmc_summary.json profiles/pmc_$k.json || exit 1; done
bash tools/evidence.sh r05_final4/ev || exit $?
}

r05_ah() {
# r05_ah: the first-dispatched tile rows cast by half footprints (32 rays per wave): SVO_HALF_ROWS 0 (the final build's
# layout) / 4 / 8 / 16 — parity of the primary casts on h8, A/B C3 / C4 / C5 / shaded
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ah; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_h8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=3 bash tools/ab_lib.sh r05_ah_c3 variants/libsvo_h0.so variants/libsvo_h4.so variants/libsvo_h8.so variants/libsvo_h16.so || exit 1
REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r05_ah_c5 variants/libsvo_h0.so variants/libsvo_h4.so variants/libsvo_h8.so variants/libsvo_h16.so || exit 1
REPS=2 BENCH_ARGS="--ao 16" bash tools/ab_lib.sh r05_ah_ao variants/libsvo_h0.so variants/libsvo_h4.so variants/libsvo_h8.so variants/libsvo_h16.so || exit 1
REPS=2 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_ah_sh variants/libsvo_h0.so variants/libsvo_h4.so variants/libsvo_h8.so variants/libsvo_h16.so || exit 1
}

r05_ai() {
# r05_ai: the frame schedule sorted every 4th scheduled frame (se4) against the final build (ae = aedae530) — the
# schedule and shading suites on se4, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ai; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_se4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_shade.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_ai_sh variants/libsvo_ae.so variants/libsvo_se4.so || exit 1
}

r05_aj() {
# r05_aj: the frame schedule sorted every 4th frame and used only near the camera it was sorted from (se4b) against the
# final build (ae) — schedule / shading suites on se4b, A/B shaded C3, and both under camera motion (tools/shade_motion.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_aj; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_se4b.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_shade.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_aj_sh variants/libsvo_ae.so variants/libsvo_se4b.so || exit 1
for v in ae se4b; do
SVO_LIB=$PWD/variants/libsvo_$v.so timeout -k 10 300 python tools/shade_motion.py > $OUT/motion_$v.txt 2>&1 || { tail $OUT/motion_$v.txt; exit 1; }
echo "== $v"; tail -8 $OUT/motion_$v.txt
done
}

r05_final5() {
# r05_final5: the final build (the schedule sorted every 4th frame): the GPU suite,
# smoke, every config's PMC passes (copied into this box's profiles/ so the bench lines read them), then tools/evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_final5; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
echo "[r05_final5] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_all.sh r05_pmc5 || exit $?
for k in c3 c3f c3_ao16 c5 c3_shade c2; do cp gpurun_out/r05_pmc5_$k/pmc_summary.json profiles/pmc_$k.json || exit 1; done
bash tools/evidence.sh r05_final5/ev || exit $?
}

r05_ak() {
# r05_ak: the depth-14 shading parity test (7-level tree: the launch-sized LDS path at its deepest)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ak; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shade.py -k "depth14 or depth12" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
}

r05_al() {
# r05_al: shadow rays on every ceiling level of the solid tree (CEIL 4: its quads) instead of its 16 / 64 pair (sq)
# against the final build (f5 = 0e9fff53) — shading suites on sq, A/B shaded C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_al; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_sq.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_schedule.py tests/test_gpu_bridge.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
REPS=4 BENCH_ARGS="--shade" bash tools/ab_lib.sh r05_al_sh variants/libsvo_f5.so variants/libsvo_sq.so || exit 1
}

r05_am() {
# r05_am: the round's last tree — the full GPU suite (with the depth-14 shading test), smoke, the shaded frame's parts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_am; mkdir -p $OUT
sha256sum raytracing_test_amd/libsvo_rt.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python tools/shade_parts.py > $OUT/shade_parts.txt 2>&1 || { tail $OUT/shade_parts.txt; exit 1; }
cat $OUT/shade_parts.txt
}

r05_an() {
# r05_an: half footprints (32 rays per wave) for the first SVO_HALF_ROWS local tile rows of launches with tile_row_step
# >= 4 only (strong-scaling shards; full frames unchanged): sh8 / sh16 / sh1000 (every row) — a verified 4-rank gloo
# strong run on sh1000, then the one-GPU shard curves at N = 4 / 8 for the product build and each variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_an; mkdir -p $OUT
SVO_LIB=$PWD/variants/libsvo_sh1000.so timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --frames 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/g4.json 2> $OUT/g4.err || { tail -20 $OUT/g4.err; exit 1; }
grep '^{' $OUT/g4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('g4 strong verified', d.get('gather_verified'))"
for v in default sh8 sh16 sh1000; do
  if [ $v = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/variants/libsvo_$v.so; fi
  for c in c3 c5; do
    timeout -k 10 300 python tools/shard_curve.py --config $c --ns 1,4,8 --reps 15 > $OUT/shard_${c}_$v.json 2> $OUT/shard_${c}_$v.err || { tail $OUT/shard_${c}_$v.err; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/shard_${c}_$v.json') if l.startswith('{')][-1])
for e in d['curve']: print('$v', '$c', e['n'], e['max_us'], [round(x,1) for x in e['rank_us']])"
  done
done
}

r05_ao() {
# r05_ao: the product build with half footprints for small launches (a wave budget: strong-scaling shards) — the full GPU
# suite, the shard curves (C3 / C5, N = 1, 2, 4, 8), the C3 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ao; mkdir -p $OUT
sha256sum raytracing_test_amd/libsvo_rt.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; }
for c in c3 c5; do
  timeout -k 10 300 python tools/shard_curve.py --config $c --ns 1,2,4,8 > $OUT/shard_$c.json 2> $OUT/shard_$c.err || { tail $OUT/shard_$c.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/shard_$c.json') if l.startswith('{')][-1])
for e in d['curve']: print('$c', e['n'], e['max_us'], e['ideal_us'], e.get('inflight_max_us'), [round(x,1) for x in e['rank_us']])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit 1
grep '^{' $OUT/c3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}

r05_final6() {
# r05_final6: the final build (half footprints for small launches): the GPU suite,
# smoke, every config's PMC passes (copied into this box's profiles/ so the bench lines read them), then tools/evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_final6; mkdir -p $OUT; export TMPDIR=/tmp
sha256sum raytracing_test_amd/libsvo_rt.so
echo "[r05_final6] $(date +%T) pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_all.sh r05_pmc6 || exit $?
for k in c3 c3f c3_ao16 c5 c3_shade c2; do cp gpurun_out/r05_pmc6_$k/pmc_summary.json profiles/pmc_$k.json || exit 1; done
bash tools/evidence.sh r05_final6/ev || exit $?
}

r05_ap() {
# r05_ap: the default bench line and the shaded one with the round's last bench.py (sanity)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_ap; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/shade.json 2> $OUT/shade.err || { tail $OUT/shade.err; exit 1; }
for n in c3 shade; do grep '^{' $OUT/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$n', d['ms_per_step'], r.get('avg_launch_ms'), r.get('counters','')[:60], d['config'].get('dispatch_order','')[:90])"; done
}

name=${1:?usage: r05_index.sh <session name: a b c d e f g h i j k l m n o p q r s t u v w x y z aa pmc final ab ac ad ae final3 af ag final4 ah ai aj final5 ak al am an ao final6 ap>}
shift
case " a b c d e f g h i j k l m n o p q r s t u v w x y z aa pmc final ab ac ad ae final3 af ag final4 ah ai aj final5 ak al am an ao final6 ap " in *" $name "*) "r05_$name" "$@" ;; *) echo "no session r05_$name" >&2; exit 2 ;; esac
