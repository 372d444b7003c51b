set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_vision_ops_gpu.py tests/test_bn_gpu.py tests/test_grad_sink_gpu.py > gpurun_out/tv.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/tv.log | head -30; exit 1; }
timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn.json 2> gpurun_out/rn.err || exit 1
DTF_CONV_GEMM_DW=never timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn_never.json 2> gpurun_out/rn_never.err || exit 1
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/bert128.json 2> gpurun_out/bert128.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_rn2 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rn_p.json 2> gpurun_out/rn_p.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_bert128 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/bert128_p.json 2> gpurun_out/bert128_p.err
