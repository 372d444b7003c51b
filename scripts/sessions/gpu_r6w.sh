#!/bin/bash
# round 6, session w: BERT-base tied word gradient: the fused embedding scatters into the
# decoder dW (no zeroed table, no autograd add): transformer / op / model tests, then same-box A/B vs ab_old/ (HEAD)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_transformer_gpu.py tests/test_ops_gpu.py tests/test_models_gpu.py -k "bert or embed or xent or transformer or layernorm or gelu or attn or dropout" > $OUT/w_tests.log 2>&1; rc=$?
tail -2 $OUT/w_tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  local v=$1; local d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
  (cd $d && timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > $OUT/w_bert_$v.log 2>&1) || { tail -5 $OUT/w_bert_$v.log; exit 1; }
  echo "bert $v $(grep -h '^{' $OUT/w_bert_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run new; run old; done
