set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r5p_gpu_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r5p_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5p_lr2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5p_lr2.log
timeout -k 10 300 python scripts/bench_graph_step.py 2000 > gpurun_out/r5p_graph_step.log 2>&1 || { tail -n 20 gpurun_out/r5p_graph_step.log; exit 1; }
tail -n 1 gpurun_out/r5p_graph_step.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5p_bench.log 2>&1 || { tail -n 20 gpurun_out/r5p_bench.log; exit 1; }
tail -n 1 gpurun_out/r5p_bench.log | cut -c1-300
timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5p_resnet.log 2>&1 || { tail -n 20 gpurun_out/r5p_resnet.log; exit 1; }
grep '^{' gpurun_out/r5p_resnet.log | tail -n 1 | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_r5p -o lr2 -- python3 scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5p_lr2_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn10 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/r5p_rn_prof.json 2> gpurun_out/r5p_rn_prof.err || exit 1
db=$(find /tmp/prof_rn10 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 70 > gpurun_out/r5p_rn_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5p_rn_steps.txt
echo done
