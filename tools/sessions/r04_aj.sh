#!/bin/bash
# r04 session AJ: PMC passes of C4 (the 8-wave AO instance) and C5 at the round's build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/pmc.sh r04_aj/pmc_c4 --ao 16 > gpurun_out/r04_aj_c4.log 2>&1 || { tail gpurun_out/r04_aj_c4.log; exit 1; }
tail -4 gpurun_out/r04_aj_c4.log
bash tools/pmc.sh r04_aj/pmc_c5 --config c5 > gpurun_out/r04_aj_c5.log 2>&1 || { tail gpurun_out/r04_aj_c5.log; exit 1; }
tail -4 gpurun_out/r04_aj_c5.log
