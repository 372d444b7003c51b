set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_mlp_persist_gpu.py tests/test_resident_gpu.py tests/test_lowering_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5q_tests.log 2>&1 || { tail -n 30 gpurun_out/r5q_tests.log; exit 1; }
tail -n 1 gpurun_out/r5q_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5q_bench$i.log 2>&1 || { tail -n 20 gpurun_out/r5q_bench$i.log; exit 1; }
  tail -n 1 gpurun_out/r5q_bench$i.log | cut -c1-260
done
timeout -k 10 300 python scripts/bench_graph_step.py 2000 > gpurun_out/r5q_graph_step.log 2>&1 || { tail -n 20 gpurun_out/r5q_graph_step.log; exit 1; }
tail -n 1 gpurun_out/r5q_graph_step.log | cut -c1-300
echo done
