# bench.py at the driver's short setting (x3) and the same-GPU 2-rank bench test
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20_$i.log 2>&1 || exit 1; grep '^{' gpurun_out/b20_$i.log | cut -c1-220; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_mlp_persist_gpu.py -k "bench_two_ranks" > gpurun_out/t_bench2.log 2>&1; rc=$?; tail -2 gpurun_out/t_bench2.log; exit $rc
