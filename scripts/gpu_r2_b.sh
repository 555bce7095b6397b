#!/bin/bash
# Round 2, call b: new dgrad kernel + TP emulation + golden tests; native step A/B of the dgrad forms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_emulation_gpu.py tests/test_golden_gpu.py tests/test_graphs_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/r2b_tests.log | head -30; tail -30 gpurun_out/r2b_tests.log; exit 1; }
tail -2 gpurun_out/r2b_tests.log
timeout -k 10 300 python scripts/native_ab.py --tp 1 2 4 8 --variants 8=0 8=1 --rounds 3 --epochs 3 > gpurun_out/r2b_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2b_native_ab.txt; exit 1; }
cat gpurun_out/r2b_native_ab.txt
