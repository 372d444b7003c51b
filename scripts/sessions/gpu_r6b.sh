#!/bin/bash
# round 6, session b: the sharded tables on the IPC data plane (2 / 4 ranks on
# cuda:0 == 1 rank), Wide&Deep at N = 1 and N = 2 same-GPU, and the
# reference loop's per-run time at 1 worker (resident) for comparison
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_sharded_ipc_gpu.py > $OUT/sharded_ipc.log 2>&1; rc=$?
echo "[sharded_ipc] rc=$rc"; tail -3 $OUT/sharded_ipc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_models.py --model wide_deep --graph --steps 100 --warmup 10 > $OUT/wd_n1.log 2>&1; rc=$?
echo "[wd_n1] rc=$rc"; tail -1 $OUT/wd_n1.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 \
  scripts/bench_models.py --model wide_deep --steps 100 --warmup 10 > $OUT/wd_n2.log 2>&1; rc=$?
echo "[wd_n2] rc=$rc"; grep '^{' $OUT/wd_n2.log | tail -1 | cut -c1-900; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29534 \
  scripts/bench_models.py --model wide_deep --graph --steps 100 --warmup 10 > $OUT/wd_n2_graph.log 2>&1; rc=$?
echo "[wd_n2_graph] rc=$rc"; grep '^{' $OUT/wd_n2_graph.log | tail -1 | cut -c1-900; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_graph_step.py --workers 1 1000 > $OUT/bench_workers1.log 2>&1; rc=$?
echo "[workers1] rc=$rc"; tail -1 $OUT/bench_workers1.log; exit $rc
