set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02f; mkdir -p $OUT; export TMPDIR=/tmp
SVO_STAMPS=$OUT/stamps_c3.npy SVO_RAY_WORK=$OUT/work_c3.npy timeout -k 10 300 python bench.py --stats --no-cpu-baseline --steps 5 > $OUT/b.json 2> $OUT/b.err; echo rc=$?
SVO_STAMPS=$OUT/stamps_c5.npy timeout -k 10 300 python bench.py --stats --no-cpu-baseline --steps 5 --config c5 > $OUT/b5.json 2> $OUT/b5.err; echo rc=$?
grep timeline $OUT/*.err | cut -c1-400
