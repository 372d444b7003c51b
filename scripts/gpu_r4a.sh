set -o pipefail
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_mlp_gemm_gpu.py > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; grep -E "Error|assert|FAIL" gpurun_out/t1.log | head -30; exit 1; }
for B in 1024 4096; do timeout -k 10 200 python -u bench.py --batch $B --steps 500 --warmup 50 > gpurun_out/bg_$B.json 2> gpurun_out/bg_$B.err || exit 1; done
timeout -k 10 200 python -u bench.py --batch 4096 --steps 500 --warmup 50 --prefetch side > gpurun_out/bg_4096s.json 2> gpurun_out/bg_4096s.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g4096 -o run -- python3 bench.py --batch 4096 --steps 200 --warmup 20 > gpurun_out/pg_4096.json 2> gpurun_out/pg_4096.err
