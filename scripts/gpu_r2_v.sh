#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2v_tests.log 2>&1; rc=$?
grep -E "FAILED|^E " gpurun_out/r2v_tests.log | head -20; tail -2 gpurun_out/r2v_tests.log
exit $rc
