# r06 final, part 2: with the final build's PMC summaries in profiles/ (part 1), every config's bench line, the N > 1
# rehearsals (gloo, the RCCL stand-in), the watchdog test and the rocprofv3 kernel traces (tools/evidence.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
sha256sum raytracing_test_amd/libsvo_rt.so
bash tools/evidence.sh r06_final2 || exit $?
