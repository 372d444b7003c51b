set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_resident_gpu.py tests/test_lowering_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1 || { tail -n 30 gpurun_out/r5c_tests.log; exit 1; }
tail -n 2 gpurun_out/r5c_tests.log
timeout -k 10 300 python scripts/bench_graph_step.py 2000 > gpurun_out/r5c_graph_step.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5c_graph_step.log
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5c_lr2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5c_lr2.log
DTF_SLR_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_general -o lr2 -- python scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5c_lr2_general_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_fused -o lr2 -- python scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5c_lr2_fused_prof.log 2>&1 || exit 1
echo done
