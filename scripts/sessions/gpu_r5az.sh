set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r5az_gpu_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r5az_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5az_smoke.log 2>&1 || { tail -n 20 gpurun_out/r5az_smoke.log; exit 1; }
tail -n 1 gpurun_out/r5az_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5az_bench.log 2>&1 || { tail -n 20 gpurun_out/r5az_bench.log; exit 1; }
tail -n 1 gpurun_out/r5az_bench.log | cut -c1-300
timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5az_bert.json 2> gpurun_out/r5az_bert.err || { tail -n 20 gpurun_out/r5az_bert.err; exit 1; }
tail -n 1 gpurun_out/r5az_bert.json | cut -c1-200
timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5az_resnet.log 2>&1 || { tail -n 20 gpurun_out/r5az_resnet.log; exit 1; }
grep '^{' gpurun_out/r5az_resnet.log | tail -n 1 | cut -c1-140
echo done
