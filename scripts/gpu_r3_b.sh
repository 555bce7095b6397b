#!/bin/bash
# Round 3, call B: the in-launch hand-offs with batched sc1 loads (fused head, dgrad slab
# reduction, folded fc1 epilogue) against the launch-per-stage chain, through the native
# executor at every TP shard (1-rank peer-mapped stand-in).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "head or dgrad or wgrad" \
  > gpurun_out/r3b_kernel_tests.log 2>&1 || { tail -40 gpurun_out/r3b_kernel_tests.log; exit 1; }
tail -2 gpurun_out/r3b_kernel_tests.log
$T 400 python -u scripts/native_ab.py --tp 1 2 4 8 --allreduce ipc --variants "21=1,22=1,23=1" "22=1,23=1" "21=1,23=1" "21=1,22=1" 21=0 \
  --rounds 5 --epochs 4 > gpurun_out/r3b_handoff_ab.txt 2>&1 || { tail -20 gpurun_out/r3b_handoff_ab.txt; exit 1; }
cat gpurun_out/r3b_handoff_ab.txt
