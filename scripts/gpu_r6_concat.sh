#!/bin/bash
# round 6: ws = 9 concat bench A/B over the streaming wgrad's run length (variant 22) on one box,
# and the concat TP = 8 shard stand-in (wgbench concat_tp8); output under gpurun_out/r6c
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6c
mkdir -p $O
for v in -1 4 8 16 -1 4 8 16; do
  timeout -k 10 300 python bench.py --mode concat --world_size 9 --steps 1 --warmup 1 --kernel_variant 22=$v > $O/concat_$v.json 2> $O/concat_$v.err || { echo CBENCH_FAIL; tail $O/concat_$v.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/concat_$v.json').read().strip().splitlines()[-1]); print('concat ws9 v22=$v', r['value'], r['ms_per_step'], r['config']['phase_seconds'])" | tee -a $O/bench_ab.txt
done
for v in -1 2 4 8 -1 2 4 8; do
  timeout -k 10 120 python scripts/wgbench.py --case concat_tp8 --iters 50 --variant 22=$v >> $O/wgbench_concat_tp8.txt 2>&1 || { echo WGB_FAIL; tail $O/wgbench_concat_tp8.txt; exit 1; }
done
grep variants $O/wgbench_concat_tp8.txt
