# N-rank in-kernel exchange modes (one-shot vs two-shot) with ranks sharing one GPU:
# bit-identity selftests, then bench.py's exchange tuning line at N=2 and N=3.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -le 1 ]; }
run pytest_xmode 600 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_mlp_persist_gpu.py -k "multi_rank_same_gpu or two_ranks" &&
DTF_BENCH_SAME_GPU=1 run b2same 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 bench.py --gpus 2 --steps 500 --warmup 50 &&
DTF_BENCH_SAME_GPU=1 run b3same 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr=127.0.0.1 --master-port=29612 bench.py --gpus 3 --steps 500 --warmup 50
