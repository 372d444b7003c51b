#!/bin/bash
# round 6, session m: BN elementwise passes with per-thread coefficients
# (hoisted out of the grid-stride loop, several chunks per thread): BN / conv
# tests, ResNet-50 at DTF_BN_EW_ITERS 4 / 1 (= the old shape) / 8, and a
# graphed Wide&Deep run on the reverted (merge-sort) build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_bn_gpu.py tests/test_conv_igemm_gpu.py tests/test_grad_sink_gpu.py > $OUT/m_tests.log 2>&1; rc=$?
tail -2 $OUT/m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_models.py --model wide_deep --graph --steps 200 --warmup 20 > $OUT/m_wd.log 2>&1 || { tail -5 $OUT/m_wd.log; exit 1; }
echo "wd $(grep -h '^{' $OUT/m_wd.log | cut -c100-200)"
for v in 4 1 4 1 8; do
  DTF_BN_EW_ITERS=$v timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > $OUT/m_resnet_$v.log 2>&1 || { tail -n 20 $OUT/m_resnet_$v.log; exit 1; }
  echo "resnet iters=$v $(grep -h '^{' $OUT/m_resnet_$v.log | cut -c60-200)"
done
