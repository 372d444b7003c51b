#!/bin/bash
# round 6, session n: wave index through readfirstlane in conv_igemm /
# attention / gemm.hip: their GPU tests, then same-box A/B vs ab_old/ (HEAD):
# ResNet-50, BERT-base, Wide&Deep graphed, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_conv_igemm_gpu.py tests/test_ops_gpu.py tests/test_transformer_gpu.py tests/test_models_gpu.py > $OUT/n_tests.log 2>&1; rc=$?
tail -2 $OUT/n_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # variant model args...
  local v=$1 m=$2; shift 2; local d=$ROOT; [ $v = old ] && d=$ROOT/ab_old
  (cd $d && timeout -k 10 400 python scripts/bench_models.py --model $m "$@" > $OUT/n_${m}_$v.log 2>&1) || { tail -5 $OUT/n_${m}_$v.log; exit 1; }
  echo "$m $v $(grep -h '^{' $OUT/n_${m}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for i in 1 2; do
  run new resnet50 --steps 30 --warmup 10; run old resnet50 --steps 30 --warmup 10
done
for i in 1 2; do
  run new bert_base --batch 128 --steps 30 --warmup 10; run old bert_base --batch 128 --steps 30 --warmup 10
done
run new wide_deep --graph --steps 200 --warmup 20; run old wide_deep --graph --steps 200 --warmup 20
