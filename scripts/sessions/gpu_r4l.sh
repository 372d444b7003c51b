set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_bn_gpu.py tests/test_vision_ops_gpu.py tests/test_transformer_gpu.py tests/test_gemm_dgelu_gpu.py tests/test_grad_sink_gpu.py > gpurun_out/tl.log 2>&1 || { grep -E "Error|assert|FAIL|error" gpurun_out/tl.log | head -30; exit 1; }
timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn_l.json 2> gpurun_out/rn_l.err || exit 1
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/bert_l.json 2> gpurun_out/bert_l.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn4 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rn_p.json 2> gpurun_out/rn_p.err || exit 1
db=$(find /tmp/prof_rn4 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/rn4_steps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_bert4 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/bert_p.json 2> gpurun_out/bert_p.err || exit 1
db=$(find /tmp/prof_bert4 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/bert4_steps.txt 2>&1
