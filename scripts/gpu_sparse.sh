# Sparse path on the GPU: route/philox kernels, sparse+W&D model tests, the lr2
# product configuration (F=1e9, B=500, lr 1) with init/memory numbers, and a
# steady-state kernel trace (init excluded via the spin marker).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -le 1 ]; }
run pytest_sparse 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_ops_gpu.py tests/test_models_gpu.py -k "route or philox or sparse or wide or embedding or graphed" &&
run lr2 300 python scripts/bench_models.py --model lr2 --steps 500 --warmup 50 &&
run lr2g 300 python scripts/bench_models.py --model lr2 --steps 2000 --warmup 50 --graph &&
run wd 300 python scripts/bench_models.py --model wide_deep --steps 100 --warmup 10 &&
run rp_lr2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_lr2 -o rp -- python scripts/bench_models.py --model lr2 --steps 200 --warmup 20 --trace-marker --graph &&
run rp_wd 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_wd -o rp -- python scripts/bench_models.py --model wide_deep --steps 50 --warmup 10 --trace-marker
