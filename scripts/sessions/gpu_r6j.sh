#!/bin/bash
# round 6, session j: BERT-base with the FFN1 input gradient moved to gemm_big
# (DTF_BIG_GEMM_SET, alternating with the round-5 table on the same box) and
# ResNet-50 after the 64-wide transposed-image swizzle
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
for i in 1 2; do
  for v in base flip; do
    set_=""; [ $v = flip ] && set_="dx:16384:768:3072=1"
    DTF_BIG_GEMM_SET=$set_ timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > $OUT/j_bert_${v}_$i.json 2> $OUT/j_bert_${v}_$i.err || { tail -n 20 $OUT/j_bert_${v}_$i.err; exit 1; }
    echo "bert $v $i $(grep -h '^{' $OUT/j_bert_${v}_$i.json | cut -c1-200)"
  done
done
for i in 1 2; do
  timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > $OUT/j_resnet_$i.log 2>&1 || { tail -n 20 $OUT/j_resnet_$i.log; exit 1; }
  echo "resnet $i $(grep -h '^{' $OUT/j_resnet_$i.log | cut -c1-200)"
done
