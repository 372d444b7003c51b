#!/bin/bash
# round 6, session u: ResNet-50 kernel trace after the no-gather projections (what glue is left)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
rm -rf /tmp/prof_resnet6
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_resnet6 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > $OUT/t_resnet_prof.json 2> $OUT/t_resnet_prof.err || exit 1
db=$(find /tmp/prof_resnet6 -name "*_results.db" | head -n 1); python scripts/rocpd_steps.py $db --steps 8 --top 60 > $OUT/t_resnet_steps.txt 2>&1
python scripts/kernel_shares.py $OUT/t_resnet_steps.txt > $OUT/t_resnet_shares.txt 2>&1
head -3 $OUT/t_resnet_steps.txt; cat $OUT/t_resnet_shares.txt
