set -o pipefail
timeout -k 10 100 python -u -m pytest -q --timeout 60 tests/test_mlp_gemm_gpu.py > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; grep -E "Error|assert|FAIL" gpurun_out/t1.log | head -30; exit 1; }
timeout -k 10 200 python -u scripts/probes/mlpg_stages.py > gpurun_out/stages.log 2>&1 || exit 1
for B in 1024 4096; do for P in serial side; do timeout -k 10 200 python -u bench.py --batch $B --steps 1000 --warmup 50 --prefetch $P > gpurun_out/bg_${B}_$P.json 2> gpurun_out/bg_${B}_$P.err || exit 1; done; done
