set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_vision_ops_gpu.py tests/test_bn_gpu.py > gpurun_out/tv.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/tv.log | head -30; exit 1; }
timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn_fold.json 2> gpurun_out/rn_fold.err || exit 1
DTF_RES_FOLD=0 timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn_nofold.json 2> gpurun_out/rn_nofold.err || exit 1
timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn_fold2.json 2> gpurun_out/rn_fold2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn3 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 --trace-marker > gpurun_out/rn_p.json 2> gpurun_out/rn_p.err || exit 1
db=$(find /tmp/prof_rn3 -name "*_results.db"); python scripts/rocpd_summary.py $db gpurun_out/rn3_kernels.csv --after spin > gpurun_out/rn3_sum.log 2>&1
