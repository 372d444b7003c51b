set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_vision_ops_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5aq_tests.log 2>&1 || { tail -n 40 gpurun_out/r5aq_tests.log; exit 1; }
DTF_CONV_FWD_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5aq_tests_fwdxcd.log 2>&1 || { tail -n 40 gpurun_out/r5aq_tests_fwdxcd.log; exit 1; }
tail -n 1 gpurun_out/r5aq_tests_fwdxcd.log
tail -n 1 gpurun_out/r5aq_tests.log
for x in 1 0; do
  DTF_CONV_XCD=$x timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5aq_wgrad_xcd$x.jsonl 2>&1 || { tail -n 20 gpurun_out/r5aq_wgrad_xcd$x.jsonl; exit 1; }
done
python - <<'PY'
import json
a = [json.loads(l) for l in open("gpurun_out/r5aq_wgrad_xcd1.jsonl") if l.startswith("{")]
b = [json.loads(l) for l in open("gpurun_out/r5aq_wgrad_xcd0.jsonl") if l.startswith("{")]
for x, y in zip(a, b):
    print((x["ks"], x["C"], x["K"], x["H"], x["stride"]), "xcd", x["igemm_us"], "plain", y["igemm_us"], "miopen", x.get("miopen_us"))
PY
for v in "1 0" "0 0" "1 1" "1 0"; do
  set -- $v
  DTF_CONV_XCD=$1 DTF_CONV_FWD_XCD=$2 timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5aq_resnet_$1$2.log 2>&1 || { tail -n 20 gpurun_out/r5aq_resnet_$1$2.log; exit 1; }
  echo "wgrad_xcd=$1 fwd_xcd=$2 $(grep '^{' gpurun_out/r5aq_resnet_$1$2.log | tail -n 1 | cut -c1-140)"
done
echo done
