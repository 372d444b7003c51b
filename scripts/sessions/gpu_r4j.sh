set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gemm_dgelu_gpu.py tests/test_gemm_big_gpu.py tests/test_transformer_gpu.py tests/test_grad_sink_gpu.py > gpurun_out/tdg.log 2>&1 || { grep -E "Error|assert|FAIL|error" gpurun_out/tdg.log | head -30; exit 1; }
B="python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/bert_ga$i.json 2> gpurun_out/bert_ga$i.err || exit 1
DTF_GEMM_DGELU=bwd timeout -k 10 300 $B > gpurun_out/bert_dg$i.json 2> gpurun_out/bert_dg$i.err || exit 1
DTF_GEMM_DGELU=0 timeout -k 10 300 $B > gpurun_out/bert_nodg$i.json 2> gpurun_out/bert_nodg$i.err || exit 1
done
