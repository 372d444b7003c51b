#!/bin/bash
# round 6, session ae: ln_bwd with 16-byte accesses, half a wave per row
# (DTF_LN16_BWD=1, a knob of that build; kernel since removed) vs the 8-byte kernel: LN / BERT
# tests, isolated kernel times, then same-box BERT-base alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
DTF_LN16_BWD=1 timeout -k 10 600 $PYT -x tests/test_transformer_gpu.py -k "bdrln or layernorm or bert or embed or mask" > $OUT/ae_tests.log 2>&1; rc=$?
tail -2 $OUT/ae_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $OUT/ae_ln.jsonl
for i in 1 2; do
  for v in 1 0; do
    DTF_LN16_BWD=$v timeout -k 10 120 python scripts/probes/ln_kernels_time.py | sed "s/\"tree\": \"repo\"/\"ln16\": $v/" >> $OUT/ae_ln.jsonl 2> $OUT/ae_ln_$v.err || { tail -5 $OUT/ae_ln_$v.err; exit 1; }
  done
done
cat $OUT/ae_ln.jsonl
run() {
  local v=$1
  DTF_LN16_BWD=$v timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > $OUT/ae_bert_$v.log 2>&1 || { tail -5 $OUT/ae_bert_$v.log; exit 1; }
  echo "bert ln16_bwd=$v $(grep -h '^{' $OUT/ae_bert_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run 1; run 0; done
