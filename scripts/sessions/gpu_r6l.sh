#!/bin/bash
# round 6, session l: resident Session engine with its per-run stamps compiled
# only into the instrumented build: resident tests, bench_graph_step x2, stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_resident_gpu.py tests/test_compat_ipc_gpu.py > $OUT/l_tests.log 2>&1; rc=$?
tail -3 $OUT/l_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_graph_step.py 2000 > $OUT/l_graph_step_$i.json 2> $OUT/l_graph_step_$i.err || exit $?
  cut -c1-400 $OUT/l_graph_step_$i.json
done
timeout -k 10 300 python -u scripts/prof_resident.py > $OUT/l_res_stamps.json 2> $OUT/l_res_stamps.err || exit $?
cut -c1-600 $OUT/l_res_stamps.json
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $OUT/l_bench_$i.log 2>&1 || exit $?
  grep -h '^{' $OUT/l_bench_$i.log | cut -c120-260
done
