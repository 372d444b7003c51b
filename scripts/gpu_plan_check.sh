cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_persist_gpu.py -k "f32 or fp32 or short_timed or bench" > gpurun_out/t_plan.log 2>&1 || { tail -30 gpurun_out/t_plan.log; exit 1; }
tail -1 gpurun_out/t_plan.log
timeout -k 10 120 python scripts/probes/launch_overhead.py > gpurun_out/launch_overhead.log 2>&1 || exit 1
tail -1 gpurun_out/launch_overhead.log
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20_$i.log 2>&1 || exit 1; grep '^{' gpurun_out/b20_$i.log | cut -c1-200; done
