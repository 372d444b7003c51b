#!/bin/bash
# round 6, session i: R = 64 transposed-image swizzle (gemm_big 192-wide B_q1,
# conv_igemm 64-wide tiles): GEMM / conv numerics tests, layout probe + PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_gemm_big_gpu.py tests/test_conv_igemm_gpu.py > $OUT/i_tests.log 2>&1; rc=$?
tail -3 $OUT/i_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probes/gemm_layout_ab.py > $OUT/i_layout.jsonl 2> $OUT/i_layout.err || exit $?
cat $OUT/i_layout.jsonl
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum"
rm -rf $OUT/i_pmc_nc
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $OUT/i_pmc_nc -o run -- \
  python3 scripts/probes/gemm_layout_ab.py pmc nc 16384 768 3072 > $OUT/i_pmc_nc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/i_pmc_nc/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "gemm_8ph" in row.get("Kernel_Name", ""):
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
print("nc", {k: round(sum(v) / len(v), 0) for k, v in agg.items()})
PY
