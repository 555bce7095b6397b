#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_golden_gpu.py tests/test_tp_emulation_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r2h_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2h_tests.log | head -30; tail -2 gpurun_out/r2h_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/native_ab.py --tp 1 2 4 8 --variants 12=0 12=1 --rounds 3 --epochs 3 > gpurun_out/r2h_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2h_native_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2h_native_ab.txt
