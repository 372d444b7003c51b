# rocprofv3 kernel stats of the fused-attention probe (tuning)
set -e
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
rm -rf gpurun_out/prof_attn
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn -o run -- python3 scripts/probes/attn_dropout_cost.py > gpurun_out/prof_attn.log 2>&1
echo ok
