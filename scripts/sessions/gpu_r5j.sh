set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
# pytest rc 1 = test failures (keep going); anything else (crash / timeout) stops the script
t() { timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 150 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc; }
t tests/test_resident_gpu.py > gpurun_out/r5j_res_alone.log 2>&1; tail -n 1 gpurun_out/r5j_res_alone.log
t tests/test_models_gpu.py tests/test_resident_gpu.py > gpurun_out/r5j_res_after_models.log 2>&1; tail -n 1 gpurun_out/r5j_res_after_models.log
t tests/test_lowering_gpu.py tests/test_resident_gpu.py > gpurun_out/r5j_res_after_lowering.log 2>&1; tail -n 1 gpurun_out/r5j_res_after_lowering.log
t tests/test_bn_gpu.py tests/test_conv_igemm_gpu.py > gpurun_out/r5j_bn.log 2>&1; tail -n 1 gpurun_out/r5j_bn.log
for feed in direct stage dma; do
  DTF_SLR_FEED=$feed timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5j_lr2_$feed.log 2>&1 || { tail -n 20 gpurun_out/r5j_lr2_$feed.log; exit 1; }
  tail -n 1 gpurun_out/r5j_lr2_$feed.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_direct -o lr2 -- python3 scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5j_lr2_prof.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5j_resnet.log 2>&1 || { tail -n 20 gpurun_out/r5j_resnet.log; exit 1; }
grep '^{' gpurun_out/r5j_resnet.log | tail -n 1
echo done
