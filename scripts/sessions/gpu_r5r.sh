set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_resident_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5r_tests.log 2>&1 || { tail -n 30 gpurun_out/r5r_tests.log; exit 1; }
tail -n 1 gpurun_out/r5r_tests.log
timeout -k 10 300 python scripts/bench_graph_step.py 2000 > gpurun_out/r5r_graph_step.log 2>&1 || { tail -n 20 gpurun_out/r5r_graph_step.log; exit 1; }
tail -n 1 gpurun_out/r5r_graph_step.log | cut -c1-300
timeout -k 10 300 python scripts/prof_persist_f32.py fp32 > gpurun_out/r5r_phases.log 2>&1 || { tail -n 30 gpurun_out/r5r_phases.log; exit 1; }
grep -A12 launch_stamps gpurun_out/r5r_phases.log | head -14
grep -A4 '"launch_20"' gpurun_out/r5r_phases.log
echo done
