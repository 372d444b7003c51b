set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_lowering_gpu.py tests/test_ops_gpu.py > gpurun_out/tlow.log 2>&1 || { grep -E "Error|assert|FAIL|error" gpurun_out/tlow.log | head -30; exit 1; }
timeout -k 10 400 python -u scripts/bench_graph_step.py 2000 > gpurun_out/bgs.json 2> gpurun_out/bgs.err || exit 1
timeout -k 10 400 python -u scripts/bench_graph_step.py 2000 > gpurun_out/bgs2.json 2> gpurun_out/bgs2.err || exit 1
