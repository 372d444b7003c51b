set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_vision_ops_gpu.py tests/test_grad_sink_gpu.py tests/test_ddp_gpu.py > gpurun_out/tr.log 2>&1 || { grep -E "Error|assert|FAIL|error" gpurun_out/tr.log | head -30; exit 1; }
B="python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/rn_cl$i.json 2> gpurun_out/rn_cl$i.err || exit 1
DTF_CONV_SINK_CL=0 timeout -k 10 300 $B > gpurun_out/rn_nocl$i.json 2> gpurun_out/rn_nocl$i.err || exit 1
done
