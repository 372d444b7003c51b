# Host-side wait strategy A/B for the headline's short timed run: the HIP
# runtime spins ROC_ACTIVE_WAIT_TIMEOUT us on a completion signal before it
# sleeps on an interrupt.  Runs scripts/probes/launch_overhead.py and
# bench.py --steps 20 --warmup 5 with the default and with a long spin.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for t in default 2000; do
  if [ "$t" = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$t; fi
  timeout -k 10 200 python scripts/probes/launch_overhead.py > gpurun_out/launch_overhead_$t.log 2>&1 || exit $?
  echo "[launch_overhead $t]"; tail -1 gpurun_out/launch_overhead_$t.log
  for i in 1 2 3; do
    timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_wait_${t}_$i.log 2>&1 || exit $?
    grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"step_time_p50_ms": [0-9.]*' gpurun_out/bench_wait_${t}_$i.log | tr '\n' ' '; echo
  done
done
