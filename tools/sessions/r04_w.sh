#!/bin/bash
# r04 session W: PMC passes of the shading pass at the working tree (profiles/pmc_c3_shade.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/pmc.sh r04_w_pmc_shade --shade
