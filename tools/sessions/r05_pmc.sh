#!/bin/bash
# r05_pmc: PMC passes of every bench config on the product build (commit 9f8e7ae's library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
sha256sum raytracing_test_amd/libsvo_rt.so
bash tools/pmc_all.sh r05_pmc || exit $?
