#!/bin/bash
# round 6, session q: ResNet-50's stride-2 1x1 projections without the gathered
# copy (DTF_CONV_S2_GATHER=0: forward / weight gradient on the implicit GEMM's
# strided loads, chosen per shape against MIOpen): conv tests, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_conv_igemm_gpu.py tests/test_bn_gpu.py > $OUT/q_tests.log 2>&1; rc=$?
tail -2 $OUT/q_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    DTF_CONV_S2_GATHER=$v timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > $OUT/q_resnet_${v}_$i.log 2>&1 || { tail -n 20 $OUT/q_resnet_${v}_$i.log; exit 1; }
    echo "resnet gather=$v $(grep -h '^{' $OUT/q_resnet_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
