#!/bin/bash
# round 6, session ag: BERT-base and ResNet-50 at the final round-6 build, two runs each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
rm -f $OUT/ag_models.jsonl
for i in 1 2; do
  for m in bert_base resnet50; do
    timeout -k 10 400 python scripts/bench_models.py --model $m --batch 128 --steps 30 --warmup 10 > $OUT/ag_$m.log 2>&1 || { tail -5 $OUT/ag_$m.log; exit 1; }
    grep -h '^{' $OUT/ag_$m.log >> $OUT/ag_models.jsonl
    echo "$m $(grep -h '^{' $OUT/ag_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], d.get("final_loss"))')"
  done
done
