#!/bin/bash
# float4 slab reductions (variant 9) and the small-K dgrad split (variant 5 = 8 restores S = 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "dgrad or linear_fwd" -q --timeout 200 --timeout-method thread > gpurun_out/r2o_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2o_tests.log | head -30; tail -2 gpurun_out/r2o_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/native_ab.py --tp 1 2 4 8 --variants 9=0 9=1 --rounds 3 --epochs 3 > gpurun_out/r2o_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2o_native_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2o_native_ab.txt
