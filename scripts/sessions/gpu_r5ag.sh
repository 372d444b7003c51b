set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn20 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/r5ag_rn_prof.json 2> gpurun_out/r5ag_rn_prof.err || exit 1
db=$(find /tmp/prof_rn20 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 20 --context templated > gpurun_out/r5ag_rn_steps.txt 2>&1
python scripts/rocpd_steps.py $db --steps 8 --top 5 --context strided_add > gpurun_out/r5ag_rn_steps2.txt 2>&1
sed -n '/--- kernels around/,$p' gpurun_out/r5ag_rn_steps.txt | cut -c1-130
echo done
