#!/bin/bash
# Round 3, call I: the IPC server head with wave 0's W3 loads after its flag wait: per-step
# times at TP 2 / 4 / 8 (1-rank peer-mapped stand-in) and the multi-process TP tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u scripts/native_ab.py --tp 2 4 8 --variants chain=0 --allreduce ipc --rounds 5 --epochs 3 > gpurun_out/r3i_ipc_head_order.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r3i_ipc_head_order.txt
[ $rc -eq 0 ] || exit $rc
$T 400 python -u -m pytest tests/test_tp_processes_gpu.py tests/test_ipc_allreduce_gpu.py tests/test_tp_emulation_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3i_tests.txt
exit $rc
