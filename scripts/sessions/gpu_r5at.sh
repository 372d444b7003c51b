set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 16384 65536 4096 16384 65536; do
  DTF_BN_EW_CAP=$c timeout -k 10 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5at_resnet_$c.log 2>&1 || { tail -n 20 gpurun_out/r5at_resnet_$c.log; exit 1; }
  echo "cap=$c $(grep '^{' gpurun_out/r5at_resnet_$c.log | tail -n 1 | cut -c1-120)"
done
echo done
