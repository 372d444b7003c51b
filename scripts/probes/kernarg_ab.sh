#!/bin/bash
# Headline engine launch prologue: kernel arguments in device memory
# (HIP_FORCE_DEV_KERNARG=1) vs the runtime default -- launch stamps
# (scripts/prof_persist_f32.py) and the driver-shape 20-step bench, each twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
for v in default 1 0; do
  if [ $v = default ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 180 python -u scripts/prof_persist_f32.py fp32 > $OUT/kernarg_$v.json 2> $OUT/kernarg_$v.err || exit $?
  for i in 1 2; do
    timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $OUT/kernarg_bench_${v}_$i.log 2>&1 || exit $?
  done
  echo "kernarg $v: $(python3 -c "import json,sys;t=open('$OUT/kernarg_$v.json').read();d=json.loads(t[t.index('{'):]);print(d['launch_stamps_us'], d['launch_20'], d['step_us_median'])")"
  grep -h '^{' $OUT/kernarg_bench_${v}_*.log | cut -c150-330
done
