#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_golden_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r2g_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2g_tests.log | head -40; tail -2 gpurun_out/r2g_tests.log
[ $rc -le 1 ] || exit $rc
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --mode ushape --steps 2 --warmup 1 --dtype $dt --num_samples 20000 > gpurun_out/r2g_ushape_$dt.json 2>&1 || { echo U_FAIL; tail -5 gpurun_out/r2g_ushape_$dt.json; exit 1; }
  tail -1 gpurun_out/r2g_ushape_$dt.json | cut -c1-260
done
for B in 32 64; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --batch_size $B --server_epochs 1 > gpurun_out/r2g_sisa_b$B.json 2>&1 || { echo B_FAIL; tail -5 gpurun_out/r2g_sisa_b$B.json; exit 1; }
  tail -1 gpurun_out/r2g_sisa_b$B.json | cut -c1-260
done
