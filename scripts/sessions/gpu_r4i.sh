set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/rn_sink$i.json 2> gpurun_out/rn_sink$i.err || exit 1
DTF_CONV_SINK_CL=0 timeout -k 10 300 $B > gpurun_out/rn_nosink$i.json 2> gpurun_out/rn_nosink$i.err || exit 1
done
