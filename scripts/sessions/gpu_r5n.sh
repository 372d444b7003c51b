set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r5n_gpu_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r5n_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr2_r5n -o lr2 -- python3 scripts/bench_lr2_compat.py --steps 100 > gpurun_out/r5n_lr2_prof.log 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5n_lr2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r5n_lr2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5n_bench.log 2>&1 || { tail -n 20 gpurun_out/r5n_bench.log; exit 1; }
tail -n 1 gpurun_out/r5n_bench.log | cut -c1-300
echo done
