set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn3 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rn_p.json 2> gpurun_out/rn_p.err || exit 1
db=$(find /tmp/prof_rn3 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/rn3_steps.txt 2>&1
