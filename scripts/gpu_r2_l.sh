#!/bin/bash
# MFMA head_fwd (variant 15): numerics, graph-replay probe, native executor A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "server_head3 or linear_fwd_partial" -q --timeout 120 --timeout-method thread > gpurun_out/r2l_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2l_tests.log | head -30; tail -2 gpurun_out/r2l_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./scripts/probe/head_probe > gpurun_out/r2l_head_probe.txt 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r2l_head_probe.txt; exit 1; }
head -12 gpurun_out/r2l_head_probe.txt
timeout -k 10 300 python scripts/native_ab.py --tp 1 8 --variants 15=0 15=1 "15=1,14=1" --rounds 3 --epochs 3 > gpurun_out/r2l_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2l_native_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2l_native_ab.txt
