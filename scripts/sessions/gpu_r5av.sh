set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_bn_gpu.py tests/test_vision_ops_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5av_tests.log 2>&1 || { tail -n 40 gpurun_out/r5av_tests.log; exit 1; }
tail -n 1 gpurun_out/r5av_tests.log
for f in 1 0 1 0; do
  DTF_BN_FUSED_FIN=$f timeout -k 10 240 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5av_resnet_$f.log 2>&1 || { tail -n 20 gpurun_out/r5av_resnet_$f.log; exit 1; }
  echo "fused_fin=$f $(grep '^{' gpurun_out/r5av_resnet_$f.log | tail -n 1 | cut -c1-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn28 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/r5av_rn_prof.json 2> gpurun_out/r5av_rn_prof.err || exit 1
db=$(find /tmp/prof_rn28 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 90 > gpurun_out/r5av_rn_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5av_rn_steps.txt
grep -h "fin_apply\|bwd_finalize\|bn_bwd_apply" gpurun_out/r5av_rn_steps.txt | cut -c1-100
echo done
