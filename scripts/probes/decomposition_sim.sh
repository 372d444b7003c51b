#!/bin/bash
# Headline engine: what the 14-workgroup (7 hidden blocks x 2 feature slices) and
# 7-workgroup (7 x 1, no E1) decompositions would cost, measured on the
# 28-workgroup engine with each workgroup's work scaled to theirs (DTF_PERSIST_EXP
# 2 / 4, csrc/kernels/mlp_persist_f32.hip compute<EXP>): phase stamps
# (scripts/prof_persist_f32.py) and the driver-shape 20-step bench per mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
for e in 0 2 4; do
  DTF_PERSIST_EXP=$e timeout -k 10 180 python -u scripts/prof_persist_f32.py fp32 > $OUT/decomp_exp$e.json 2> $OUT/decomp_exp$e.err || exit $?
  for i in 1 2; do
    DTF_PERSIST_EXP=$e timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $OUT/decomp_bench_exp${e}_$i.log 2>&1 || exit $?
  done
  echo "exp $e: step_us_median $(grep step_us_median $OUT/decomp_exp$e.json)"
  grep -h '^{' $OUT/decomp_bench_exp${e}_*.log | cut -c1-330
done
