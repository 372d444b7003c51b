#!/bin/bash
# Same-box A/B of the headline engine: this tree vs ab_old/ (a copy built from
# HEAD's mlp_persist_f32.hip), alternating, launch stamps + driver-shape benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
for i in 1 2 3; do
  for v in new old; do
    d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
    (cd $d && timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $OUT/ab_${v}_$i.log 2>&1) || exit $?
    echo "$v $i $(grep -h '^{' $OUT/ab_${v}_$i.log | cut -c120-260)"
  done
done
for v in new old; do
  d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
  (cd $d && timeout -k 10 180 python -u scripts/prof_persist_f32.py fp32 > $OUT/ab_prof_$v.json 2> $OUT/ab_prof_$v.err) || exit $?
  python3 -c "import json;t=open('$OUT/ab_prof_$v.json').read();d=json.loads(t[t.index('{'):]);print('$v', d['launch_stamps_us'], d['launch_20'], d['step_us_median'], d['segments_us_median_p90'])"
done
