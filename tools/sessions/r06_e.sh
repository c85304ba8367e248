# r06 session e: where the shaded frame's time goes on the current build (its own block durations, the parts)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_e; mkdir -p $O
timeout -k 10 300 python tools/shade_critical.py > $O/shade_critical.json 2> $O/shade_critical.err; echo "critical rc=$?" >> $O/steps.log
timeout -k 10 300 python tools/shade_parts.py > $O/shade_parts.txt 2> $O/shade_parts.err; echo "parts rc=$?" >> $O/steps.log
cat $O/shade_critical.json $O/shade_parts.txt $O/steps.log; tail -3 $O/shade_critical.err
