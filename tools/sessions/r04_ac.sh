#!/bin/bash
# r04 session AC: the AO instance with its hemisphere table read from the kernel arguments instead of LDS (the LDS then
# allows 8 waves): 7 (71 VGPRs) and 8 waves (64 VGPRs, 4 spilled) against HEAD's 6; C4 at 16 and 20 samples
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPS=4 BENCH_ARGS="--ao 16" timeout -k 10 600 bash tools/ab_lib.sh r04_ac/ao16 variants/libsvo_base.so variants/libsvo_ao7.so variants/libsvo_ao8.so || exit 1
REPS=3 BENCH_ARGS="--ao 20" timeout -k 10 600 bash tools/ab_lib.sh r04_ac/ao20 variants/libsvo_base.so variants/libsvo_ao7.so variants/libsvo_ao8.so || exit 1
