# Compat-graph lowering on the GPU: lowering tests, then the graph-mode MNIST
# example (no --fused) under a rocprofv3 kernel trace (kernels per step).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -le 1 ]; }
PORT=$((20000 + RANDOM % 20000))
run pytest_lowering 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_lowering_gpu.py tests/test_lowering_cpu.py tests/test_meta_graph_cpu.py "tests/test_mlp_persist_gpu.py::test_bench_two_ranks_same_gpu_short_run" &&
run rp_graph 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_graph -o rp -- python examples/mnist_example.py --job_name=worker --task_index=0 --ps_hosts= --worker_hosts=127.0.0.1:$PORT --max_steps=500 --train_size=20000 --learning_rate=0.1 --logs_path=/tmp/logs_graph --frequency=100 --result_json=gpurun_out/graph_example.json &&
run graph_plain 300 python examples/mnist_example.py --job_name=worker --task_index=0 --ps_hosts= --worker_hosts=127.0.0.1:$((PORT + 1)) --max_steps=2000 --train_size=55000 --learning_rate=0.1 --logs_path=/tmp/logs_graph2 --frequency=500 &&
run bench_graph 200 python scripts/bench_graph_step.py 2000
