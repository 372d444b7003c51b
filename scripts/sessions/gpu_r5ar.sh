set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_vision_ops_gpu.py tests/test_bn_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5ar_tests.log 2>&1 || { tail -n 40 gpurun_out/r5ar_tests.log; exit 1; }
tail -n 1 gpurun_out/r5ar_tests.log
timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5ar_wgrad.jsonl 2>&1 || { tail -n 20 gpurun_out/r5ar_wgrad.jsonl; exit 1; }
cut -c50-200 gpurun_out/r5ar_wgrad.jsonl
for i in 1 2; do
  timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5ar_resnet$i.log 2>&1 || { tail -n 20 gpurun_out/r5ar_resnet$i.log; exit 1; }
  echo "run$i $(grep '^{' gpurun_out/r5ar_resnet$i.log | tail -n 1 | cut -c1-140)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn26 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/r5ar_rn_prof.json 2> gpurun_out/r5ar_rn_prof.err || exit 1
db=$(find /tmp/prof_rn26 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 90 > gpurun_out/r5ar_rn_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5ar_rn_steps.txt
echo done
