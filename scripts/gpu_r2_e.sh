#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tp_emulation_gpu.py tests/test_golden_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|^E " gpurun_out/r2e_tests.log | head -40; tail -2 gpurun_out/r2e_tests.log
exit $rc
