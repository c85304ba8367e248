#!/bin/bash
# r05_y: the product build with the split shading trace (camera octant, CEIL 1, 6 waves): full GPU suite, shaded and
# plain C3 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --shade --no-cpu-baseline > $OUT/shade.json 2>$OUT/shade.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c3.json 2>$OUT/c3.err || exit 1
python3 -c "
import json
for n in ('shade','c3'):
    d=json.loads([l for l in open('$OUT/%s.json'%n) if l.startswith('{')][-1]); r=d.get('roofline') or {}
    print(n, d['ms_per_step'], r.get('avg_launch_ms'))"
