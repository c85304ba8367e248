#!/bin/bash
# r04 session BE: PMC passes of the shading instance with the frame schedule (warmup 3: the timed launches scheduled)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/pmc.sh r04_be/pmc_shade --shade --warmup 3 > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04_be/pmc_shade/pmc_summary.json')); print({k: d[k] for k in ('hbm_bytes_per_launch', 'l2_hit_rate', 'valu_per_wave', 'salu_per_wave', 'bench_avg_launch_ms') if k in d})"
