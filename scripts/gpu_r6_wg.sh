#!/bin/bash
# round 6: the streaming wgrad form (variant 22 = row tiles per workgroup): bitwise test, then
# wgbench A/B over the concat / vanilla / U-shape layer groups, then concat ws = 9 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_wg
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for case in concat vanilla ushape; do
  for v in 0 2 4 8 16 0 4 8; do
    timeout -k 10 120 python scripts/wgbench.py --case $case --iters 30 --variant 22=$v >> $O/wgbench.txt 2>&1 || { echo WGB_FAIL; tail $O/wgbench.txt; exit 1; }
  done
done
grep variants $O/wgbench.txt
for v in 0 8 0 8; do
  timeout -k 10 300 python bench.py --mode concat --world_size 9 --steps 1 --warmup 1 --kernel_variant 22=$v > $O/concat_$v.json 2> $O/concat_$v.err || { echo CBENCH_FAIL; tail $O/concat_$v.err; exit 1; }
  python -c "import json,sys; r=json.loads(open('$O/concat_$v.json').read().strip().splitlines()[-1]); print('concat v22=$v', r['value'], r['ms_per_step'])" | tee -a $O/concat_ab.txt
done
