#!/bin/bash
# Round-4 GPU iteration: hybrid tests + A/B, remote split epochs, NT GEMM bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4/hy_tests.log 2>&1 || { echo HY_TEST_FAIL; grep -E "PASS|FAIL|Error|assert" gpurun_out/r4/hy_tests.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/r4/hy_tests.log
timeout -k 10 300 python scripts/hybrid_ab.py --tp 1 2 4 --steps 400 --rounds 3 --trace \
  > gpurun_out/r4/hy_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r4/hy_ab.log; exit 1; }
grep -v amdgpu gpurun_out/r4/hy_ab.log | grep -E "median|per-workgroup|trace wg 0"
timeout -k 10 700 python -u -m pytest tests/test_split_remote_gpu.py tests/test_split_native_gpu.py \
  -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/split_tests.log 2>&1 \
  || { echo SPLIT_TEST_FAIL; grep -E "PASS|FAIL|Error|assert|rank" gpurun_out/r4/split_tests.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/r4/split_tests.log
timeout -k 10 200 python scripts/gemm_bench.py --reps 6 > gpurun_out/r4/gemm_nt.log 2>&1 || echo GEMM_FAIL
grep -v amdgpu gpurun_out/r4/gemm_nt.log | tail -24
