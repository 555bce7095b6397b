#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "server_head3 or linear_fwd" -q --timeout 120 --timeout-method thread > gpurun_out/r2m_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2m_tests.log | head -30; tail -2 gpurun_out/r2m_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./scripts/probe/head_probe > gpurun_out/r2m_probe.txt 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r2m_probe.txt; exit 1; }
cat gpurun_out/r2m_probe.txt
