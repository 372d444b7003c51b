set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5y_tests.log 2>&1 || { tail -n 40 gpurun_out/r5y_tests.log; exit 1; }
tail -n 1 gpurun_out/r5y_tests.log
timeout -k 10 300 python scripts/probes/conv_bnb_epilogue.py > gpurun_out/r5y_bnb_probe.jsonl 2>&1 || { tail -n 20 gpurun_out/r5y_bnb_probe.jsonl; exit 1; }
cat gpurun_out/r5y_bnb_probe.jsonl
for e in 1 0; do
  DTF_BN_BWD_EPILOGUE=$e timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5y_resnet_epi$e.log 2>&1 || { tail -n 20 gpurun_out/r5y_resnet_epi$e.log; exit 1; }
  echo "epi=$e $(grep '^{' gpurun_out/r5y_resnet_epi$e.log | tail -n 1 | cut -c1-160)"
done
echo done
