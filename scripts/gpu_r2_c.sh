#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tp_emulation_gpu.py tests/test_golden_gpu.py tests/test_graphs_gpu.py tests/test_kernels_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|^E " gpurun_out/r2c_tests.log | grep -v "PASSED" | head -40; tail -3 gpurun_out/r2c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/native_ab.py --tp 1 2 4 8 --variants 8=0 8=1 --rounds 3 --epochs 3 > gpurun_out/r2c_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2c_native_ab.txt; exit 1; }
cat gpurun_out/r2c_native_ab.txt
