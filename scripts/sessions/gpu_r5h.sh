set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_bn_gpu.py tests/test_models_gpu.py tests/test_lowering_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5h_tests.log 2>&1 || { tail -n 40 gpurun_out/r5h_tests.log; exit 1; }
tail -n 2 gpurun_out/r5h_tests.log
timeout -k 10 300 python scripts/probes/conv3x3_paths.py > gpurun_out/r5h_conv3x3.log 2>&1 || { tail -n 20 gpurun_out/r5h_conv3x3.log; exit 1; }
grep '^{' gpurun_out/r5h_conv3x3.log
for mode in auto never; do
  DTF_CONV_IGEMM=$mode timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5h_resnet_$mode.log 2>&1 || { tail -n 20 gpurun_out/r5h_resnet_$mode.log; exit 1; }
  grep '^{' gpurun_out/r5h_resnet_$mode.log | tail -n 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn7 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/r5h_rn_prof.json 2> gpurun_out/r5h_rn_prof.err || exit 1
db=$(find /tmp/prof_rn7 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/r5h_rn_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5h_rn_steps.txt
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5h_bert.json 2> gpurun_out/r5h_bert.err || exit 1
tail -n 1 gpurun_out/r5h_bert.json
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_bert7 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/r5h_bert_prof.json 2> gpurun_out/r5h_bert_prof.err || exit 1
db=$(find /tmp/prof_bert7 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/r5h_bert_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5h_bert_steps.txt
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5h_lr2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5h_lr2.log
echo done
