#!/bin/bash
# round 6, session y: ln_bwd with the next row's s / dy / statistics prefetched
# (a wave walks ~4 rows): LN tests, isolated kernel times new vs ab_old/ (HEAD),
# then same-box BERT-base A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_transformer_gpu.py -k "ln or layernorm or bert or embed" > $OUT/y_tests.log 2>&1; rc=$?
tail -2 $OUT/y_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
    (cd $d && timeout -k 10 120 python scripts/probes/ln_kernels_time.py) >> $OUT/y_ln.jsonl 2>$OUT/y_ln_$v.err || { tail -5 $OUT/y_ln_$v.err; exit 1; }
  done
done
cat $OUT/y_ln.jsonl
run() {
  local v=$1; local d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
  (cd $d && timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > $OUT/y_bert_$v.log 2>&1) || { tail -5 $OUT/y_bert_$v.log; exit 1; }
  echo "bert $v $(grep -h '^{' $OUT/y_bert_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run new; run old; done
