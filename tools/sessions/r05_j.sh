#!/bin/bash
# r05_j: the top tile rows alone (tools/tail_probe.py) on each ceiling layout: does a finer / coarser layout shorten the
# far-field critical path although it slows the whole frame?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05_j; mkdir -p $OUT
for v in default k1s2 k2s2 k1s3; do
  if [ $v = default ]; then unset SVO_LIB; else export SVO_LIB=$PWD/variants/libsvo_$v.so; fi
  timeout -k 10 200 python tools/tail_probe.py --reps 10 > $OUT/tail_$v.txt 2>/dev/null || exit 1
  echo "$v $(tail -1 $OUT/tail_$v.txt)"
done
