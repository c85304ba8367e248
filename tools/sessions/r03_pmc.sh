#!/bin/bash
# r03 PMC passes of every config on the final build (tools/pmc_all.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/pmc_all.sh r03pmc4
