set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 20 --warmup 10 > gpurun_out/r5t_resnet.log 2>&1 || { tail -n 20 gpurun_out/r5t_resnet.log; exit 1; }
grep '^{' gpurun_out/r5t_resnet.log | tail -n 1 | cut -c1-200
echo done
