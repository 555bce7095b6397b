#!/bin/bash
# round 6: ws = 9 concat bench over the pinned row count (variant 23: -1 off, 0 the default), interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_pin3
mkdir -p $O
for v in -1 0 384 -1 0 384 -1 0 384; do
  timeout -k 10 300 python bench.py --mode concat --world_size 9 --steps 3 --warmup 1 --kernel_variant 23=$v > $O/concat_$v.json 2> $O/concat_$v.err || { echo CBENCH_FAIL; tail $O/concat_$v.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/concat_$v.json').read().strip().splitlines()[-1]); print('concat ws9 v23=$v', r['value'], r['ms_per_step'], r['config']['phase_seconds'])" | tee -a $O/bench_ab.txt
done
