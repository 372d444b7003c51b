set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 150 --timeout-method thread -k "weight_gradient or shadow or flip" > gpurun_out/r5ae_tests.log 2>&1 || { tail -n 40 gpurun_out/r5ae_tests.log; exit 1; }
tail -n 1 gpurun_out/r5ae_tests.log
timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5ae_wgrad_512.jsonl 2>&1 || { tail -n 20 gpurun_out/r5ae_wgrad_512.jsonl; exit 1; }
for w in 128 256 1024; do
  DTF_CONV_WGRAD_WGS=$w timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5ae_wgrad_$w.jsonl 2>&1 || { tail -n 20 gpurun_out/r5ae_wgrad_$w.jsonl; exit 1; }
done
python - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/r5ae_wgrad_*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); k = (d["ks"], d["C"], d["K"], d["H"], d["stride"])
            rows.setdefault(k, {})[f"{d['wgs']}"] = d["igemm_us"]
            if "miopen_us" in d: rows[k]["miopen"] = d["miopen_us"]
for k, v in rows.items(): print(k, v)
PY
