set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_transformer_gpu.py tests/test_grad_sink_gpu.py tests/test_gemm_dgelu_gpu.py > gpurun_out/tn.log 2>&1 || { grep -E "Error|assert|FAIL|error" gpurun_out/tn.log | head -30; exit 1; }
B="python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/bert_n$i.json 2> gpurun_out/bert_n$i.err || exit 1
DTF_ATTN_BIAS_PARTIALS=0 timeout -k 10 300 $B > gpurun_out/bert_no$i.json 2> gpurun_out/bert_no$i.err || exit 1
done
