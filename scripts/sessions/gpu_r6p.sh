#!/bin/bash
# round 6, session p: resident Session engine at the final headline build:
# bench_graph_step x2 + per-run stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_graph_step.py 2000 > $OUT/p_graph_step_$i.json 2> $OUT/p_graph_step_$i.err || exit $?
  cut -c1-300 $OUT/p_graph_step_$i.json
done
timeout -k 10 300 python -u scripts/prof_resident.py > $OUT/p_res_stamps.json 2> $OUT/p_res_stamps.err || exit $?
cut -c1-600 $OUT/p_res_stamps.json
