#!/bin/bash
# round 6, session r: no-gather strided 1x1 as the default -- conv / BN / model /
# sink GPU tests, ResNet-50 x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_conv_igemm_gpu.py tests/test_bn_gpu.py tests/test_models_gpu.py tests/test_grad_sink_gpu.py tests/test_ddp_gpu.py > $OUT/r_tests.log 2>&1; rc=$?
tail -2 $OUT/r_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > $OUT/r_resnet_$i.log 2>&1 || { tail -n 20 $OUT/r_resnet_$i.log; exit 1; }
  grep -h '^{' $OUT/r_resnet_$i.log | cut -c1-300
done
