set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "wave_order or multi_frame or sharding" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for o in none "feedback --order-group 1" "feedback --order-group 4" "feedback --order-group 16" "feedback --order-group 60"; do
  tag=$(echo $o | tr -d ' -')
  timeout -k 10 120 python bench.py --no-cpu-baseline --order $o --steps 40 > $OUT/b_${tag}_$rep.json 2>> $OUT/b.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/b_${tag}_$rep.json').read()); print('$o', d['ms_per_step'], d['roofline']['avg_launch_ms'], round(d['value']/1e9,3))"
done; done
for o in none; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --order $o --config c5 --steps 20 > $OUT/b5_$o.json 2>> $OUT/b.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/b5_$o.json').read()); print('c5 $o', d['ms_per_step'], d['roofline']['avg_launch_ms'], round(d['value']/1e9,3))"
  timeout -k 10 120 python bench.py --no-cpu-baseline --order $o --ao 16 --steps 20 > $OUT/b4_$o.json 2>> $OUT/b.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/b4_$o.json').read()); print('c4 $o', d['ms_per_step'], d['roofline']['avg_launch_ms'], round(d['value']/1e9,3))"
done
SVO_STAMPS=$OUT/stamps_fb.npy timeout -k 10 120 python bench.py --no-cpu-baseline --order feedback --steps 5 --stats > /dev/null 2> $OUT/stats_fb.err; grep timeline $OUT/stats_fb.err | cut -c1-400
