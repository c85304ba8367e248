#!/bin/bash
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
