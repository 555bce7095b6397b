#!/bin/bash
# round 6: selected GPU tests (argument: pytest node ids / files), log under gpurun_out/r6_tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_tests
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread "$@" > $O/tests.log 2>&1
rc=$?
echo "tests rc $rc"
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40
exit $rc
