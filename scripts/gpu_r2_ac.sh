#!/bin/bash
# U-shape head step on MFMA: numerics, U-shape bench A/B (variant 15 = 1: the FMA kernel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "head_step" -q --timeout 120 --timeout-method thread > gpurun_out/r2ac_tests.log 2>&1; rc=$?
grep -E "FAILED|^E " gpurun_out/r2ac_tests.log | head -20; tail -1 gpurun_out/r2ac_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1 0 1; do
  timeout -k 10 300 python bench.py --mode ushape --steps 3 --warmup 1 --kernel_variant 15=$v --json_out gpurun_out/r2ac_u$v.json > gpurun_out/r2ac_u$v.log 2>&1 || { echo BENCH_FAIL $v; tail -20 gpurun_out/r2ac_u$v.log; exit 1; }
  echo "15=$v $(python -c "import json;d=json.load(open('gpurun_out/r2ac_u$v.json'));print(d['value'], d['config']['phase_seconds'])")"
done
