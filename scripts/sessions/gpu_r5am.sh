set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5am_tests.log 2>&1 || { tail -n 40 gpurun_out/r5am_tests.log; exit 1; }
tail -n 1 gpurun_out/r5am_tests.log
timeout -k 10 300 python scripts/probes/conv_bnb_epilogue.py > gpurun_out/r5am_bnb_probe.jsonl 2>&1 || { tail -n 20 gpurun_out/r5am_bnb_probe.jsonl; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5am_bnb_probe.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print({k: d[k] for k in ('dy_ch','dx_ch','H','epi3_bn64_us','epi3_bn128_us','acc_bn128_us')})
"
for i in 1 2; do
  timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5am_resnet$i.log 2>&1 || { tail -n 20 gpurun_out/r5am_resnet$i.log; exit 1; }
  echo "run$i $(grep '^{' gpurun_out/r5am_resnet$i.log | tail -n 1 | cut -c1-160)"
done
echo done
