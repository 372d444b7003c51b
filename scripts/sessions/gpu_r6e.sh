#!/bin/bash
# round 6, session e: sparse routing's flat scan (no outer-dimension cumsum)
# + scatter-copy gradient packing: sharded GPU tests, W&D N = 2 same-GPU and
# N = 1 graphed, with a trace of the N = 2 step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name] rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-700; tail -2 $OUT/$name.log | cut -c1-300
         [ $rc -eq 0 ] || exit $rc; }
step sparse_tests 900 $PYT -x tests/test_sharded_ipc_gpu.py tests/test_models_gpu.py tests/test_sparse_optim_gpu.py
step wd_n1 300 python scripts/bench_models.py --model wide_deep --graph --steps 100 --warmup 10
step wd_n2 400 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29561 \
  scripts/bench_models.py --model wide_deep --graph --steps 100 --warmup 10
step wd_n2_eager 400 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29562 \
  scripts/bench_models.py --model wide_deep --steps 100 --warmup 10
rm -rf $OUT/prof_wd2b
step prof_wd2b 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_wd2b -- \
  python3 -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29563 \
  scripts/bench_models.py --model wide_deep --steps 40 --warmup 5
for f in $(find $OUT/prof_wd2b -name "*kernel_trace.csv"); do
  echo "== $f"; python3 scripts/prof_summary.py "$f" --steps 45 --top 25 | tee -a $OUT/prof_wd2b_summary.txt | head -14
done
rm -rf $OUT/prof_wd1b
step prof_wd1b 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_wd1b -o run -- \
  python3 scripts/bench_models.py --model wide_deep --graph --steps 200 --warmup 10
f=$(find $OUT/prof_wd1b -name "*kernel_trace.csv" | head -n 1)
python3 scripts/prof_summary.py "$f" --steps 150 --tail-ms 75 --top 45 > $OUT/prof_wd1b_summary.txt; head -50 $OUT/prof_wd1b_summary.txt
step prof_resident 300 python scripts/prof_resident.py 2000
step resident_tests 300 $PYT -x tests/test_resident_gpu.py
step persist_tests 600 $PYT -x tests/test_mlp_persist_gpu.py -k "not same_gpu and not two_ranks and not eight and not five_six"
step phases 300 python scripts/prof_persist_f32.py fp32
for i in 1 2 3; do step bench20_$i 180 python bench.py --gpus 1 --steps 20 --warmup 5; done
exit 0
