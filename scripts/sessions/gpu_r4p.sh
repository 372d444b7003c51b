set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10"
timeout -k 10 300 $B > gpurun_out/rn_fm0.json 2> gpurun_out/rn_fm0.err || exit 1
MIOPEN_FIND_MODE=1 timeout -k 10 700 $B > gpurun_out/rn_fm1.json 2> gpurun_out/rn_fm1.err || exit 1
MIOPEN_FIND_MODE=1 timeout -k 10 700 $B > gpurun_out/rn_fm1b.json 2> gpurun_out/rn_fm1b.err || exit 1
