set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02j; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
for o in "" "--overlap"; do
  tag=$(echo "x$o" | tr -d ' -')
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 $o > $OUT/b_${tag}_$rep.json 2>> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${tag}_$rep.json').read()); print('$tag', d['ms_per_step'], d['roofline']['avg_launch_ms'], round(d['value']/1e9,3))"
done; done
for o in "--config c5" "--ao 16" "--shade"; do
for ov in "" "--overlap"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 $o $ov > $OUT/c.json 2>> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c.json').read()); print('$o $ov', d['ms_per_step'], d['roofline']['avg_launch_ms'], round(d['value']/1e9,3))"
done; done
