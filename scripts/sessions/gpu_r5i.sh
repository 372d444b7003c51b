set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_lowering_gpu.py tests/test_resident_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5i_tests.log 2>&1 || { tail -n 40 gpurun_out/r5i_tests.log; exit 1; }
tail -n 2 gpurun_out/r5i_tests.log
for feed in direct stage dma; do
  DTF_SLR_FEED=$feed timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5i_lr2_$feed.log 2>&1 || { tail -n 20 gpurun_out/r5i_lr2_$feed.log; exit 1; }
  tail -n 1 gpurun_out/r5i_lr2_$feed.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_direct -o lr2 -- python3 scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5i_lr2_prof.log 2>&1 || exit 1
echo done
