# split-MFMA fp32 engine iteration: numerics tests, phase profile, short + long bench (A/B vs fp32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -le 1 ]; }
run t_s28 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_persist_gpu.py -k "f32 or fp32 or s28 or short_timed" &&
run prof_s28 200 python scripts/prof_persist_f32.py fp32-s28 &&
run b20_s28 120 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp32-s28 &&
run b5500_s28 240 python bench.py --gpus 1 --precision fp32-s28 &&
run b20 120 python bench.py --gpus 1 --steps 20 --warmup 5
