# fp32 persistent engines iteration: numerics tests, phase profile, short + long bench (split default vs f32 MFMA)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -le 1 ]; }
run t_f32 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_persist_gpu.py -k "f32 or fp32 or short_timed" &&
run prof_fp32 200 python scripts/prof_persist_f32.py fp32 &&
run b20 120 python bench.py --gpus 1 --steps 20 --warmup 5 &&
run b5500 240 python bench.py --gpus 1 &&
run b20_mfma 120 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp32-mfma
