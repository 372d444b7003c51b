#!/bin/bash
# round 6, session d: Wide&Deep kernel traces -- N = 1 graphed B = 4096 (the
# verdict's re-profile) and N = 2 same-GPU (why 19 ms / step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
rm -rf $OUT/prof_wd1 $OUT/prof_wd2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_wd1 -o run -- \
  python3 scripts/bench_models.py --model wide_deep --graph --steps 30 --warmup 5 > $OUT/prof_wd1.log 2>&1
rc=$?; echo "[prof_wd1] rc=$rc"; grep '^{' $OUT/prof_wd1.log | tail -1 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof_wd1 -name "*kernel_trace.csv" | head -n 1)
python3 scripts/prof_summary.py "$f" --steps 35 --top 40 > $OUT/prof_wd1_summary.txt; head -45 $OUT/prof_wd1_summary.txt
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_wd2 -- \
  python3 -m torch.distributed.run --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29551 \
  scripts/bench_models.py --model wide_deep --steps 20 --warmup 5 > $OUT/prof_wd2.log 2>&1
rc=$?; echo "[prof_wd2] rc=$rc"; grep '^{' $OUT/prof_wd2.log | tail -1 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for f in $(find $OUT/prof_wd2 -name "*kernel_trace.csv"); do
  echo "== $f"; python3 scripts/prof_summary.py "$f" --steps 25 --top 25 | tee -a $OUT/prof_wd2_summary.txt
done
exit 0
