set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02k; mkdir -p $OUT; export TMPDIR=/tmp
for o in "" "--shade" "--ao 16" "--config c5"; do
  timeout -k 10 300 python bench.py $o > $OUT/c.json 2>> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c.json').read()); print('$o', d['ms_per_step'], (d['roofline'] or {}).get('avg_launch_ms'), round(d['value']/1e9,3), d.get('pipelined'), (d.get('cpu_baseline') or {}).get('parity_vs_gpu'))"
done
