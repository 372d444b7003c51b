set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_headline_r5 -o hl -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5ba_bench_prof.log 2>&1 || { tail -n 20 gpurun_out/r5ba_bench_prof.log; exit 1; }
tail -n 1 gpurun_out/r5ba_bench_prof.log | cut -c1-200
f=$(find gpurun_out/prof_headline_r5 -name "*kernel_stats.csv" | head -n 1); echo "$f"; head -n 8 "$f" | cut -c1-200
echo done
