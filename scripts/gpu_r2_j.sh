#!/bin/bash
# Chain pricing (variant 13 launch-skip probe) and the one-round-trip skinny forward A/B (variant 14).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "linear_fwd" -q --timeout 120 --timeout-method thread > gpurun_out/r2j_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2j_tests.log | head -30; tail -2 gpurun_out/r2j_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/native_ab.py --tp 1 8 --variants 13=0 13=1 13=2 13=4 13=8 13=16 13=15 --rounds 3 --epochs 3 > gpurun_out/r2j_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/r2j_probe.txt; exit 1; }
grep "us/step" gpurun_out/r2j_probe.txt
timeout -k 10 300 python scripts/native_ab.py --tp 1 2 4 8 --variants 14=0 14=1 --rounds 3 --epochs 3 > gpurun_out/r2j_once_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2j_once_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2j_once_ab.txt
