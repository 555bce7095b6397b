#!/bin/bash
# wgrad_group with 8-row workgroups (variant 9 = 1): numerics, then native executor A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_group" tests/test_graphs_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2u_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2u_tests.log | head -30; tail -2 gpurun_out/r2u_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/native_ab.py --tp 1 2 4 8 --variants 9=0 9=1 --rounds 3 --epochs 3 > gpurun_out/r2u_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2u_native_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2u_native_ab.txt
