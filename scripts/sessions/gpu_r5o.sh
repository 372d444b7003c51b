set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
t() { timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 150 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc; }
t tests/test_conv_igemm_gpu.py tests/test_resident_gpu.py tests/test_lowering_gpu.py > gpurun_out/r5o_tests.log 2>&1; tail -n 1 gpurun_out/r5o_tests.log
timeout -k 10 300 python scripts/bench_graph_step.py 2000 > gpurun_out/r5o_graph_step.log 2>&1 || { tail -n 20 gpurun_out/r5o_graph_step.log; exit 1; }
tail -n 1 gpurun_out/r5o_graph_step.log | cut -c1-400
timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5o_resnet.log 2>&1 || { tail -n 20 gpurun_out/r5o_resnet.log; exit 1; }
grep '^{' gpurun_out/r5o_resnet.log | tail -n 1 | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn9 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/r5o_rn_prof.json 2> gpurun_out/r5o_rn_prof.err || exit 1
db=$(find /tmp/prof_rn9 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 70 > gpurun_out/r5o_rn_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5o_rn_steps.txt
echo done
