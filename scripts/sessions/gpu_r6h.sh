#!/bin/bash
# round 6, session h: gemm_big B-layout cost (K- vs N-contiguous B at the same
# shapes, vs hipBLASLt) and PMC of both layouts at 16384 x 768 x 3072
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u scripts/probes/gemm_layout_ab.py > $OUT/h_layout.jsonl 2> $OUT/h_layout.err || exit $?
cat $OUT/h_layout.jsonl
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum"
P2="SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVES"
for lay in kc nc; do
  for p in 1 2; do
    eval cn=\$P$p
    rm -rf $OUT/h_pmc_${lay}_$p
    timeout -s KILL 90 rocprofv3 --pmc $cn --output-format csv -d $OUT/h_pmc_${lay}_$p -o run -- \
      python3 scripts/probes/gemm_layout_ab.py pmc $lay 16384 768 3072 > $OUT/h_pmc_${lay}_$p.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, collections
for lay in ("kc", "nc"):
    agg = collections.defaultdict(list)
    for p in (1, 2):
        for f in glob.glob(f"gpurun_out/h_pmc_{lay}_{p}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if "gemm_8ph" in row.get("Kernel_Name", ""):
                    agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(lay, {k: round(sum(v) / max(1, len(v) // 1), 0) for k, v in agg.items()})
PY
