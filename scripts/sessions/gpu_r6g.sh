#!/bin/bash
# round 6, session g: headline prologue without serial waits (unconditional
# buffer loads, scalars converted at the drain) -- engine tests, launch stamps,
# driver-shape benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_mlp_persist_gpu.py tests/test_resident_gpu.py > $OUT/g_tests.log 2>&1; rc=$?
tail -3 $OUT/g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u scripts/prof_persist_f32.py fp32 > $OUT/g_prof.json 2> $OUT/g_prof.err || exit $?
python3 -c "import json;t=open('$OUT/g_prof.json').read();d=json.loads(t[t.index('{'):]);print(d['launch_stamps_us'], d['launch_20'], d['step_us_median'])"
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $OUT/g_bench_$i.log 2>&1 || exit $?
  grep -h '^{' $OUT/g_bench_$i.log | cut -c1-330
done
