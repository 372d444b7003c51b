#!/bin/bash
# round 6, session c: IPC collectives with 16-byte system-coherent peer loads
# (tests again), their bandwidth vs the 8-byte atomic loads (DTF_IPC_NARROW=1),
# and Wide&Deep at N = 2 same-GPU on them
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name] rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-1500; tail -2 $OUT/$name.log | cut -c1-300
         [ $rc -eq 0 ] || exit $rc; }
step ipc_tests 600 $PYT -x tests/test_ipc_coll_gpu.py tests/test_compat_ipc_gpu.py
step bw_wide 200 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29541 scripts/probes/ipc_bw.py
DTF_IPC_NARROW=1 step bw_narrow 300 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29542 scripts/probes/ipc_bw.py
step wd_n2 400 python -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29543 \
  scripts/bench_models.py --model wide_deep --graph --steps 100 --warmup 10
exit 0
