set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for t in 1 0 1 0; do
  DTF_BIG_GEMM_TABLE=$t timeout -k 10 300 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5ay_bert_$t.json 2> gpurun_out/r5ay_bert_$t.err || { tail -n 20 gpurun_out/r5ay_bert_$t.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/r5ay_bert_$t.json').read().strip().splitlines()[-1])
n=d['config'].get('linear_gemm_native',{})
print('table=$t', d['value'], sum(1 for v in n.values() if v), '/', len(n))
"
done
echo done
