#!/bin/bash
# round 6: vanilla seam X per channel vs 8 shards (ab/run.sh), then the vanilla regression tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_seamx
mkdir -p $O
timeout -k 10 700 bash ab/run.sh > $O/ab.log 2>&1 || { echo "ab rc $?"; exit 1; }
grep -E "^== |us/step|x out|x rel" gpurun_out/ab.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vanilla_persist_gpu.py tests/test_golden_gpu.py tests/test_long_launch_gpu.py -k "vanilla" > $O/tests.log 2>&1; echo "tests rc $?"; tail -2 $O/tests.log
