set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
t() { timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 150 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc; }
for sk in priority plain; do for pre in none streams sparse; do
  DTF_RESIDENT_STREAM=$sk timeout -k 10 120 python scripts/probes/resident_relaunch.py $pre > gpurun_out/r5m_res_${sk}_$pre.log 2>&1 || { tail -n 20 gpurun_out/r5m_res_${sk}_$pre.log; exit 1; }
  echo "$sk $pre $(tail -n 1 gpurun_out/r5m_res_${sk}_$pre.log | cut -c1-220)"
done; done
t tests/test_transformer_gpu.py > gpurun_out/r5m_tfm.log 2>&1; tail -n 1 gpurun_out/r5m_tfm.log
t tests/test_models_gpu.py tests/test_resident_gpu.py > gpurun_out/r5m_models.log 2>&1; tail -n 1 gpurun_out/r5m_models.log
timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5m_lr2.log 2>&1 || { tail -n 20 gpurun_out/r5m_lr2.log; exit 1; }
tail -n 1 gpurun_out/r5m_lr2.log
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5m_bert.json 2> gpurun_out/r5m_bert.err || { tail -n 20 gpurun_out/r5m_bert.err; exit 1; }
tail -n 1 gpurun_out/r5m_bert.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_bert9 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/r5m_bert_prof.json 2> gpurun_out/r5m_bert_prof.err || exit 1
db=$(find /tmp/prof_bert9 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/r5m_bert_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5m_bert_steps.txt
grep attn gpurun_out/r5m_bert_steps.txt | cut -c1-120
echo done
