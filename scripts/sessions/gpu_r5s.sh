set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DTF_BWD_OVERLAP=1 timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_grad_sink_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5s_tests.log 2>&1 || { tail -n 30 gpurun_out/r5s_tests.log; exit 1; }
tail -n 1 gpurun_out/r5s_tests.log
for ov in 0 1 0 1; do
  DTF_BWD_OVERLAP=$ov timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5s_bert_ov$ov.json 2> gpurun_out/r5s_bert_ov$ov.err || { tail -n 20 gpurun_out/r5s_bert_ov$ov.err; exit 1; }
  echo "overlap=$ov $(tail -n 1 gpurun_out/r5s_bert_ov$ov.json | cut -c1-200)"
done
echo done
