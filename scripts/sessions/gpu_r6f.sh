#!/bin/bash
# round 6, session f/g: Wide&Deep with the fused head, sunk tower gradients and
# one-kernel input refresh: numerics (GPU vs CPU reference, graph vs eager,
# 200-step graphed regression), N = 1 / N = 2 benches and the step's trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name] rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-400; tail -2 $OUT/$name.log | cut -c1-300
         [ $rc -eq 0 ] || exit $rc; }
step wd_tests 600 $PYT -x tests/test_models_gpu.py tests/test_graph_replay_gpu.py tests/test_ops_gpu.py tests/test_sharded_ipc_gpu.py -k "wide or ipc or graph or col_sum or linear or gemm or bag"
for i in 1 2; do step wd_n1_$i 300 python scripts/bench_models.py --model wide_deep --graph --steps 200 --warmup 20; done
step wd_n2 400 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29571 \
  scripts/bench_models.py --model wide_deep --graph --steps 100 --warmup 10
rm -rf $OUT/prof_wd1c
step prof_wd1c 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_wd1c -o run -- \
  python3 scripts/bench_models.py --model wide_deep --graph --steps 200 --warmup 10
f=$(find $OUT/prof_wd1c -name "*kernel_trace.csv" | head -n 1)
python3 scripts/prof_summary.py "$f" --steps 150 --tail-ms 75 --top 45 > $OUT/prof_wd1c_summary.txt; head -30 $OUT/prof_wd1c_summary.txt
exit 0
