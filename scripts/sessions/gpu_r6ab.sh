#!/bin/bash
# round 6, session ab: conv_wgrad with three operand sets in flight (DTF_CONV_WGRAD_DEPTH=3,
# where it keeps the occupancy) vs two: conv / BN / model GPU tests at the new default,
# the per-shape weight-gradient sweep at depth 2 and 3, then ResNet-50 alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_conv_igemm_gpu.py tests/test_bn_gpu.py > $OUT/ab_tests.log 2>&1; rc=$?
tail -2 $OUT/ab_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $OUT/ab_sweep.jsonl
for d in 2 3; do
  DTF_CONV_WGRAD_DEPTH=$d timeout -k 10 300 python scripts/probes/conv_wgrad_sweep.py >> $OUT/ab_sweep.jsonl 2> $OUT/ab_sweep_$d.err || { tail -5 $OUT/ab_sweep_$d.err; exit 1; }
done
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/ab_sweep.jsonl")]
by = {}
for r in rows:
    by.setdefault((r["ks"], r["C"], r["K"], r["H"], r["stride"]), {})[r["depth"]] = r["igemm_us"]
for k, v in by.items():
    print(k, "depth2", v.get("2"), "depth3", v.get("3"))
PY
run() {
  local d=$1
  DTF_CONV_WGRAD_DEPTH=$d timeout -k 10 400 python scripts/bench_models.py --model resnet50 --batch 128 --steps 30 --warmup 10 > $OUT/ab_resnet_$d.log 2>&1 || { tail -5 $OUT/ab_resnet_$d.log; exit 1; }
  echo "resnet depth$d $(grep -h '^{' $OUT/ab_resnet_$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"
}
for i in 1 2 3; do run 3; run 2; done
