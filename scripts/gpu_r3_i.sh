#!/bin/bash
# Round 3, call I: in-tree fp32 GEMM forms (staging loads kept in registers and issued before
# the MFMAs; 32x32x2 forms) against hipBLASLt on the evaluation shapes; GEMM numerics tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "linear_fwd" > gpurun_out/r3i_tests.log 2>&1 || { tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
$T 400 python -u scripts/gemm_bench.py > gpurun_out/r3i_gemm_bench.txt 2>&1 || { tail -30 gpurun_out/r3i_gemm_bench.txt; exit 1; }
cat gpurun_out/r3i_gemm_bench.txt
