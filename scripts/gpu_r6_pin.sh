#!/bin/bash
# round 6: concat's fc1 stream with a pinned subset of rows in the Infinity Cache (variant 23 =
# rows, the rest non-temporal) -- wgbench of the concat tail step, then the ws = 9 concat bench,
# interleaved on one box.  Output under gpurun_out/r6_pin
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_pin
mkdir -p $O
for v in 0 256 384 512 0 256 384 512; do
  timeout -k 10 120 python scripts/wgbench.py --case concat --iters 30 --variant 23=$v >> $O/wgbench.txt 2>&1 || { echo WGB_FAIL; tail $O/wgbench.txt; exit 1; }
done
grep variants $O/wgbench.txt
for v in 0 384 0 384; do
  timeout -k 10 300 python bench.py --mode concat --world_size 9 --steps 1 --warmup 1 --kernel_variant 23=$v > $O/concat_$v.json 2> $O/concat_$v.err || { echo CBENCH_FAIL; tail $O/concat_$v.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/concat_$v.json').read().strip().splitlines()[-1]); print('concat ws9 v23=$v', r['value'], r['ms_per_step'], r['config']['phase_seconds'])" | tee -a $O/bench_ab.txt
done
