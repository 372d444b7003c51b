set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
t() { timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 150 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc; }
for pre in none world streams sparse; do
  timeout -k 10 120 python scripts/probes/resident_relaunch.py $pre > gpurun_out/r5l_res_$pre.log 2>&1 || { tail -n 20 gpurun_out/r5l_res_$pre.log; exit 1; }
  tail -n 1 gpurun_out/r5l_res_$pre.log
done
t tests/test_conv_igemm_gpu.py -k "handoff or stats" > gpurun_out/r5l_conv.log 2>&1; tail -n 1 gpurun_out/r5l_conv.log
for rpw in 32 16 8; do
  DTF_SLR_RPW=$rpw timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5l_lr2_rpw$rpw.log 2>&1 || { tail -n 20 gpurun_out/r5l_lr2_rpw$rpw.log; exit 1; }
  tail -n 1 gpurun_out/r5l_lr2_rpw$rpw.log
done
DTF_SLR_FEED=overlap timeout -k 10 200 python scripts/bench_lr2_compat.py > gpurun_out/r5l_lr2_overlap.log 2>&1 || { tail -n 20 gpurun_out/r5l_lr2_overlap.log; exit 1; }
tail -n 1 gpurun_out/r5l_lr2_overlap.log
echo done
