set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_bn_gpu.py tests/test_vision_ops_gpu.py > gpurun_out/tbn.log 2>&1 || { grep -E "Error|assert|FAIL|error" gpurun_out/tbn.log | head -30; exit 1; }
B="python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/rn_wg$i.json 2> gpurun_out/rn_wg$i.err || exit 1
DTF_BN_WRITE_G=0 timeout -k 10 300 $B > gpurun_out/rn_nowg$i.json 2> gpurun_out/rn_nowg$i.err || exit 1
done
