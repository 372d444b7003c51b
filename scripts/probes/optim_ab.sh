# optimizer kernel change: tests + BERT-base bench (tuning)
set -e
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_sparse_optim_gpu.py tests/test_ddp_gpu.py tests/test_bn_gpu.py tests/test_transformer_gpu.py > gpurun_out/optim_tests.log 2>&1
tail -1 gpurun_out/optim_tests.log
for i in 1 2; do
  timeout -k 10 300 python scripts/bench_models.py --model bert_base --batch 128 --steps 20 --warmup 5 > gpurun_out/bert_$i.log 2>&1
  echo "bert $(grep -o '"value": [0-9.]*' gpurun_out/bert_$i.log | head -1)"
done
