#!/bin/bash
# v13 evidence: traversal counters, SQ stall breakdown and HBM traffic PMC passes (separate passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/v13p
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --stats > gpurun_out/v13p/stats.json 2> gpurun_out/v13p/stats.err || exit 1
grep -E "stats per ray|timeline" gpurun_out/v13p/stats.err
timeout -k 10 600 bash tools/pmc_sq.sh v13sq || exit 1
timeout -k 10 600 bash tools/pmc.sh v13pmc || exit 1
