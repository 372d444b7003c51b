#!/bin/bash
# round 6, session z: colsum_partials with 16 partial-row loads in flight per thread
# (the LN backward finishing sums): LN tests, isolated kernel times new vs ab_old/ (HEAD),
# then same-box BERT-base A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_transformer_gpu.py -k "ln or layernorm or bert or embed or colsum or bias" > $OUT/z_tests.log 2>&1; rc=$?
tail -2 $OUT/z_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
    (cd $d && timeout -k 10 120 python scripts/probes/ln_kernels_time.py) >> $OUT/z_ln.jsonl 2>$OUT/z_ln_$v.err || { tail -5 $OUT/z_ln_$v.err; exit 1; }
  done
done
cat $OUT/z_ln.jsonl
run() {
  local v=$1; local d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
  (cd $d && timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > $OUT/z_bert_$v.log 2>&1) || { tail -5 $OUT/z_bert_$v.log; exit 1; }
  echo "bert $v $(grep -h '^{' $OUT/z_bert_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run new; run old; done
