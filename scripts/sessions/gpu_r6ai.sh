#!/bin/bash
# round 6, session ai: 3x3 / stride-2 max-pool with XCD-contiguous block ranges
# (DTF_POOL_XCD=1, default) vs plain order: vision-op tests, kernel times, ResNet-50 alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_vision_ops_gpu.py -k maxpool > $OUT/ai_tests.log 2>&1; rc=$?
tail -2 $OUT/ai_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $OUT/ai_pool.jsonl
for i in 1 2; do for v in 1 0; do
  DTF_POOL_XCD=$v timeout -k 10 120 python scripts/probes/maxpool_time.py >> $OUT/ai_pool.jsonl 2> $OUT/ai_pool_$v.err || { tail -5 $OUT/ai_pool_$v.err; exit 1; }
done; done
cat $OUT/ai_pool.jsonl
run() {
  local v=$1
  DTF_POOL_XCD=$v timeout -k 10 400 python scripts/bench_models.py --model resnet50 --batch 128 --steps 30 --warmup 10 > $OUT/ai_resnet_$v.log 2>&1 || { tail -5 $OUT/ai_resnet_$v.log; exit 1; }
  echo "resnet xcd=$v $(grep -h '^{' $OUT/ai_resnet_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run 1; run 0; done
