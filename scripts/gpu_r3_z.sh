#!/bin/bash
# Round 3, call Z: the chain launch with its loads in consumption order: tests, then the
# per-step A/B against the six kernels with the phase stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_chain_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3z_chain_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3z_chain_tests.txt
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/r3z_chain_tests.txt | head -20; exit 1; }
$T 400 python -u scripts/native_ab.py --tp 1 2 4 8 --variants chain=0 chain=1 --allreduce ipc --rounds 3 --epochs 2 --trace > gpurun_out/r3z_chain_ab.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r3z_chain_ab.txt | grep -v "chain phases" ; grep "chain phases" gpurun_out/r3z_chain_ab.txt | awk 'NR%3==0' | cut -c1-170
exit $rc
