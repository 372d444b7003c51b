set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5ad_wgrad_512.jsonl 2>&1 || { tail -n 20 gpurun_out/r5ad_wgrad_512.jsonl; exit 1; }
for w in 256 1024 2048; do
  DTF_CONV_WGRAD_WGS=$w timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5ad_wgrad_$w.jsonl 2>&1 || { tail -n 20 gpurun_out/r5ad_wgrad_$w.jsonl; exit 1; }
done
DTF_CONV_WGRAD_WGS=1024 DTF_CONV_WGRAD_MINSTEPS=4 timeout -k 10 200 python scripts/probes/conv_wgrad_sweep.py > gpurun_out/r5ad_wgrad_1024_m4.jsonl 2>&1 || { tail -n 20 gpurun_out/r5ad_wgrad_1024_m4.jsonl; exit 1; }
python - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/r5ad_wgrad_*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); k = (d["ks"], d["C"], d["K"], d["H"], d["stride"])
            rows.setdefault(k, {})[f"{d['wgs']}/{d['minsteps']}"] = d["igemm_us"]
            if "miopen_us" in d: rows[k]["miopen"] = d["miopen_us"]
for k, v in rows.items(): print(k, v)
PY
