set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02c; mkdir -p $OUT; export TMPDIR=/tmp
for a in "c1 --config c1" "c5 --config c5" "c2 --config c2" "c2cam0 --config c2cam0 --no-cpu-baseline"; do
  set -- $a; name=$1; shift
  echo "[r02c] $(date +%T) $name"
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; exit 1; }
done
timeout -k 10 1500 bash tools/pmc_all.sh r02c_pmc
