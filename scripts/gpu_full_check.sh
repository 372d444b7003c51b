# Full GPU validation: smoke, every GPU test, the headline bench (short + long), a rocprofv3 kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -le 1 ]; }
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" &&
run pytest_gpu 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu &&
run b20 120 python bench.py --gpus 1 --steps 20 --warmup 5 &&
run b5500 240 python bench.py --gpus 1 &&
run rp_b5500 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_b5500 -o rp -- python bench.py --gpus 1
