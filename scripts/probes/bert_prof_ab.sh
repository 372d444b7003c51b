# rocprofv3 kernel stats of BERT-base B=128 under DTF_BIG_GEMM=never / always.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for pol in never always; do
  rm -rf gpurun_out/prof_bert_$pol
  DTF_BIG_GEMM=$pol timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert_$pol -o run -- \
    python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 3 > gpurun_out/bert_prof_$pol.log 2>&1
  rc=$?; echo "[bert_prof_$pol] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bert_prof_$pol.log; exit $rc; fi
  python3 scripts/prof_summary.py gpurun_out/prof_bert_$pol/run_kernel_trace.csv --steps 13 --top 30 > gpurun_out/prof_bert_${pol}_summary.txt
  head -40 gpurun_out/prof_bert_${pol}_summary.txt
done
