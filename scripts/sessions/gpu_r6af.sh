#!/bin/bash
# round 6, session af: gemm_big slab-mode workgroup target (DTF_GEMM_SLAB_WGS: 256 default
# vs 128 / 512) on BERT-base's split-K weight gradients: GEMM tests, then BERT alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_gemm_big_gpu.py > $OUT/af_tests.log 2>&1; rc=$?
tail -2 $OUT/af_tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  local v=$1
  DTF_GEMM_SLAB_WGS=$v timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > $OUT/af_bert_$v.log 2>&1 || { tail -5 $OUT/af_bert_$v.log; exit 1; }
  echo "bert slab_wgs=$v $(grep -h '^{' $OUT/af_bert_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run 256; run 128; run 512; done
