#!/bin/bash
# round 6, session a: the IPC data plane (collectives, compat example at 2 / 4
# sync workers, per-run time of 1 ps + 2 workers) and the advisor-fix tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TESTS="tests/test_resident_gpu.py tests/test_conv_igemm_gpu.py::test_conv_bn_statistics_handoff_ignored_after_inplace_write tests/test_conv_igemm_gpu.py::test_conv_bn_statistics_handoff"
bash scripts/gpu.sh native ipc tests
