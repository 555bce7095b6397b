#!/bin/bash
# XOR-swizzled look-ahead LDS tile: bitwise check, SQ counters, native + bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/lds_layout_check.py > gpurun_out/lds_check.txt 2>&1 || { echo CHECK_FAIL; tail -20 gpurun_out/lds_check.txt; exit 1; }
cat gpurun_out/lds_check.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u scripts/native_ab.py --tp 1 8 --variants 1=0 1=2 1=1 > gpurun_out/native_ab_xor.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/native_ab_xor.txt; exit 1; }
grep "^tp=" gpurun_out/native_ab_xor.txt
for i in 1 2; do
  for v in "1=0" "1=2"; do
    timeout -k 10 200 python bench.py --mode ushape --steps 5 --warmup 2 --kernel_variant $v > gpurun_out/abx.log 2>&1 || { tail -20 gpurun_out/abx.log; exit 1; }
    python -c "import json;r=json.loads(open('gpurun_out/abx.log').read().strip().splitlines()[-1]);print('ushape','$v',r['value'],r['ms_per_step'])"
  done
done
