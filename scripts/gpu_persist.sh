#!/bin/bash
# Persistent MLP kernel: numerics tests, then the headline bench on both engines.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_persist_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/persist_tests.log 2>&1
rc=$?; tail -15 $OUT/persist_tests.log
[ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps ${STEPS:-5500} --warmup 550 > $OUT/bench_persist.log 2>&1
rc=$?; tail -2 $OUT/bench_persist.log
[ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
exit 0
