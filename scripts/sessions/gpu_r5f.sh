set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_bn_gpu.py tests/test_vision_ops_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1 || { tail -n 40 gpurun_out/r5f_tests.log; exit 1; }
tail -n 2 gpurun_out/r5f_tests.log
timeout -k 10 300 python scripts/probes/conv3x3_paths.py > gpurun_out/r5f_conv3x3.log 2>&1 || { tail -n 20 gpurun_out/r5f_conv3x3.log; exit 1; }
grep '^{' gpurun_out/r5f_conv3x3.log
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5f_lr2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5f_lr2.log
for mode in auto never; do
  DTF_CONV_IGEMM=$mode timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5f_resnet_$mode.log 2>&1 || { tail -n 20 gpurun_out/r5f_resnet_$mode.log; exit 1; }
  grep '^{' gpurun_out/r5f_resnet_$mode.log | tail -n 1
done
echo done
