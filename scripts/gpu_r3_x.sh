#!/bin/bash
# Round 3, call X: the resident epoch's phase timeline with the update / publication split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/resident_trace.py --tp 8 > gpurun_out/r3x_resident_trace.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r3x_resident_trace.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_resident_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_resident_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3x_resident_tests.txt
exit $rc
