#!/bin/bash
# PMC passes (tools/pmc.sh) of every bench config; summaries -> gpurun_out/<tag>_<key>/pmc_summary.json
# (copy to profiles/pmc_<key>.json).  usage: tools/pmc_all.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmcall}
run() { local key=$1; shift; echo "[pmc_all] $(date +%T) $key"; timeout -k 10 900 bash tools/pmc.sh ${TAG}_$key "$@" > gpurun_out/${TAG}_$key.log 2>&1; local rc=$?; echo "$key rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_$key.log; exit $rc; }; }
mkdir -p gpurun_out
run c3
run c3f --config c3f
run c3_ao16 --ao 16
run c5 --config c5
run c3_shade --shade
run c2 --config c2
