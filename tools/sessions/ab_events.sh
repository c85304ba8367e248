#!/bin/bash
# per-launch event pairs vs one pair around the timed region: ms_per_step and the launch average
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/events
for rep in 1 2 3; do
for m in "" "--region-events"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 $m > gpurun_out/events/b_${m#--}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/events/b_${m#--}_$rep.json'));print('mode=%-14s ms_per_step %.4f launch avg %.4f' % ('${m:-each}', d['ms_per_step'], d['roofline']['avg_launch_ms']))"
done
done
