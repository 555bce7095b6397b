#!/bin/bash
# Round 3, call A: peer-mapped all-reduce (release/acquire, error skipping, stalled-peer abort),
# the one-launch server head, pruned kernel variants; A/B of the fence cost and of the head
# through the native executor; then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_allreduce_gpu.py \
  tests/test_tp_processes_gpu.py -k "not bench_full" > gpurun_out/r3a_ipc_tests.log 2>&1 || { tail -40 gpurun_out/r3a_ipc_tests.log; exit 1; }
tail -5 gpurun_out/r3a_ipc_tests.log
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "head or dgrad or wgrad" \
  > gpurun_out/r3a_head_tests.log 2>&1 || { tail -40 gpurun_out/r3a_head_tests.log; exit 1; }
tail -2 gpurun_out/r3a_head_tests.log
$T 300 python -u scripts/native_ab.py --tp 1 2 4 8 --allreduce ipc --variants 21=0 21=1 22=1 23=1 "21=1,22=1,23=1" "21=0,fences=0" \
  --rounds 5 --epochs 4 > gpurun_out/r3a_head_fences_ab.txt 2>&1 || { tail -20 gpurun_out/r3a_head_fences_ab.txt; exit 1; }
cat gpurun_out/r3a_head_fences_ab.txt
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_gpu_suite.log 2>&1 || { tail -40 gpurun_out/r3a_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r3a_gpu_suite.log
