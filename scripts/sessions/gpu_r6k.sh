#!/bin/bash
# round 6, session k: headline engine with instrumentation compiled only into
# the INS instantiations (production: no stamp / knob code, 95 vs 132 SGPR
# spills): engine + resident tests, then same-box A/B vs HEAD (ab_old/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT -x tests/test_mlp_persist_gpu.py tests/test_resident_gpu.py > $OUT/k_tests.log 2>&1; rc=$?
tail -3 $OUT/k_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/probes/prologue_ab.sh
