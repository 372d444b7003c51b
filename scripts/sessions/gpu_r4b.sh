set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for B in 1024 4096; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g$B -o run -- python3 bench.py --batch $B --steps 300 --warmup 20 > gpurun_out/pg_$B.json 2> gpurun_out/pg_$B.err || exit 1
done
