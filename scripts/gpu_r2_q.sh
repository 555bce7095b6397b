#!/bin/bash
# Head kernels with DPP reductions + compile-time bf16 (variant 15 = 1: the previous kernels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_golden_gpu.py tests/test_tp_emulation_gpu.py tests/test_e2e_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r2q_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2q_tests.log | head -30; tail -2 gpurun_out/r2q_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./scripts/probe/head_probe > gpurun_out/r2q_head_probe.txt 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r2q_head_probe.txt; exit 1; }
grep -E "head_(fwd|bwd)( v0)?  |head pair( v0)?  |empty 1" gpurun_out/r2q_head_probe.txt
timeout -k 10 300 python scripts/native_ab.py --tp 1 8 --variants 15=0 15=1 --rounds 3 --epochs 3 > gpurun_out/r2q_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2q_native_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2q_native_ab.txt
