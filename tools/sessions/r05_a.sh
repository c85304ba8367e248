#!/bin/bash
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
