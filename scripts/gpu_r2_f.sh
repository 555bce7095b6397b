#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_golden_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2f_tests.log | head -40; tail -2 gpurun_out/r2f_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/r2f_gemm.txt 2>&1 || { echo GEMM_FAIL; tail gpurun_out/r2f_gemm.txt; exit 1; }
cat gpurun_out/r2f_gemm.txt
