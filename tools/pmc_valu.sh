#!/bin/bash
# VALU / SALU instructions per wave of the C3 cast kernel for library variants (one --pmc pass each):
#   tools/pmc_valu.sh <tag> <lib.so|default>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/$L; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/$TAG/$n -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/$n.log 2>&1 || { echo "$n failed"; exit 1; }
  python3 - gpurun_out/$TAG/$n "$n" <<'PY'
import csv, glob, sys, collections
d, n = sys.argv[1], sys.argv[2]
f = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(f)):
    if 'k_cast' not in r['Kernel_Name']: continue
    disp.add(r['Dispatch_Id']); acc[r['Counter_Name']] += float(r['Counter_Value'])
k = len(disp); w = acc['SQ_WAVES'] / k
print('%-18s dispatches %d  VALU/wave %.1f  SALU/wave %.1f  VMEM_RD/wave %.2f' % (n, k, acc['SQ_INSTS_VALU'] / k / w, acc['SQ_INSTS_SALU'] / k / w, acc['SQ_INSTS_VMEM_RD'] / k / w))
PY
done
