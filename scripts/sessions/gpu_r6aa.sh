#!/bin/bash
# round 6, session aa: evidence at the final headline build -- rocprofv3 kernel trace +
# stats of the driver-shape bench (20 steps), then one PMC pass (scripts/probes/pmc_headline.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
rm -rf $OUT/aa_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/aa_stats -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/aa_stats.log 2>&1 || { tail -5 $OUT/aa_stats.log; exit 1; }
grep '^{' $OUT/aa_stats.log | cut -c1-200
f=$(find $OUT/aa_stats -name "*kernel_stats.csv" | head -n 1); echo "$f"; head -8 "$f"
bash scripts/probes/pmc_headline.sh && grep '^{' gpurun_out/pmc_headline.log | cut -c1-200
f=$(find gpurun_out/pmc_headline -name "*counter_collection.csv" | head -n 1); echo "$f"; wc -l "$f"
