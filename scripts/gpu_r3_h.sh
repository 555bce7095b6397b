#!/bin/bash
# Round 3, call H: server-head kernels with the consumed-first loads (variant 6 = 0, new)
# against W3 first (6 = 1), per server step; the head / executor tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u scripts/native_ab.py --tp 1 8 --variants 6=1 6=0 --allreduce ipc --rounds 5 --epochs 3 > gpurun_out/r3h_head_order_ab.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r3h_head_order_ab.txt
[ $rc -eq 0 ] || exit $rc
$T 400 python -u -m pytest tests/test_graphs_gpu.py tests/test_golden_gpu.py tests/test_golden_modes_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3h_tests.txt
exit $rc
