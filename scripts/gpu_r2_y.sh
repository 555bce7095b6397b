#!/bin/bash
# Large-M dgrad through hipBLASLt + mask: numerics; SISA bench at batch 128 / 256.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dgrad" -q --timeout 120 --timeout-method thread > gpurun_out/r2y_tests.log 2>&1; rc=$?
grep -E "FAILED|^E " gpurun_out/r2y_tests.log | head; tail -1 gpurun_out/r2y_tests.log
[ $rc -eq 0 ] || exit $rc
for b in 128 256; do
  timeout -k 10 300 python bench.py --batch_size $b --server_epochs 1 --steps 2 --warmup 1 --json_out gpurun_out/r2y_b$b.json > gpurun_out/r2y_b$b.log 2>&1 || { echo BENCH_FAIL $b; tail -20 gpurun_out/r2y_b$b.log; exit 1; }
  tail -1 gpurun_out/r2y_b$b.log | cut -c1-200
done
