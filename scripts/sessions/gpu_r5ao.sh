set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in 0.05 0.12 0.05 0.12; do
  DTF_BIG_GEMM_MARGIN=$m timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5ao_bert_$m.json 2> gpurun_out/r5ao_bert_$m.err || { tail -n 20 gpurun_out/r5ao_bert_$m.err; exit 1; }
  python -c "
import json,sys
d=json.loads(open('gpurun_out/r5ao_bert_$m.json').read().strip().splitlines()[-1])
n=d['config'].get('linear_gemm_native',{})
print('margin=$m', d['value'], 'native:', sum(1 for v in n.values() if v), '/', len(n), [k for k,v in n.items() if not v])
"
done
DTF_BIG_GEMM_MARGIN=0.12 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_bert5 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/r5ao_bert_prof.json 2> gpurun_out/r5ao_bert_prof.err || exit 1
db=$(find /tmp/prof_bert5 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 40 > gpurun_out/r5ao_bert_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5ao_bert_steps.txt
echo done
