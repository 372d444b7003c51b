set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_models_gpu.py tests/test_lowering_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1 || { tail -n 40 gpurun_out/r5d_tests.log; exit 1; }
tail -n 2 gpurun_out/r5d_tests.log
timeout -k 10 300 python scripts/probes/conv3x3_paths.py > gpurun_out/r5d_conv3x3.log 2>&1 || { tail -n 20 gpurun_out/r5d_conv3x3.log; exit 1; }
grep '^{' gpurun_out/r5d_conv3x3.log
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5d_lr2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5d_lr2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_fused2 -o lr2 -- python scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5d_lr2_fused_prof.log 2>&1 || exit 1
echo done
