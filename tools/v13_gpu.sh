set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v13
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v13/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/v13/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
REPS=3 timeout -k 10 600 bash tools/ab_lib.sh v13lib default variants/libsvo_head.so variants/libsvo_nobox.so variants/libsvo_pack1.so variants/libsvo_novroot.so || exit 1
REPS=3 timeout -k 10 400 bash tools/ab_cfg.sh v13tile ":0" ":256" ":512" || exit 1
BENCH_ARGS="--ao 16" REPS=2 timeout -k 10 400 bash tools/ab_cfg.sh v13ao ":0" "SVO_LIB=$PWD/variants/libsvo_head.so:0" || exit 1
