#!/bin/bash
# r03 session J: finer column ceilings (16-column blocks) against the launch's critical path: parity of the
# variants, A/B on C3 / C5 / shaded, per-ray stats and the top-tile-row probe per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r03_j; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "[r03_j] $(date +%T) $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc; }
V="variants/libsvo_k2_16_256.so variants/libsvo_k2_16_64.so"
for v in $V; do n=$(basename $v .so)
  run pytest_$n 600 env SVO_LIB=$PWD/$v python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shade.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread
done
for v in default $V; do n=$(basename $v .so)
  if [ $v = default ]; then E=""; else E="SVO_LIB=$PWD/$v"; fi
  run stats_$n 300 env $E python -u bench.py --stats --steps 5 --warmup 2 --no-cpu-baseline
  run probe_$n 300 env $E python -u tools/tail_probe.py --reps 10
done
run ab_c3 900 env REPS=4 bash tools/ab_lib.sh r03_j_c3 default $V
run ab_c5 900 env REPS=2 BENCH_ARGS="--config c5" bash tools/ab_lib.sh r03_j_c5 default $V
run ab_shade 900 env REPS=2 BENCH_ARGS="--shade --pipelined-steps 0" bash tools/ab_lib.sh r03_j_sh default $V
