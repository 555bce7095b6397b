#!/bin/bash
# round 6: benches of the modes the streaming wgrad form serves (concat ws = 9 auto, vanilla
# per-batch) and the TP-shard wgbench A/B; output under gpurun_out/r6x
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6x
mkdir -p $O
for v in 0 -1 0; do
  timeout -k 10 300 python bench.py --mode concat --world_size 9 --steps 1 --warmup 1 --kernel_variant 22=$v > $O/concat_$v.json 2> $O/concat_$v.err || { echo CBENCH_FAIL; tail $O/concat_$v.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/concat_$v.json').read().strip().splitlines()[-1]); print('concat ws9 v22=$v', r['value'], r['ms_per_step'])" | tee -a $O/bench_ab.txt
done
for v in 0 -1; do
  timeout -k 10 300 python bench.py --mode vanilla --split_persist off --steps 5 --warmup 2 --kernel_variant 22=$v > $O/va_pb_$v.json 2> $O/va_pb_$v.err || { echo VBENCH_FAIL; tail $O/va_pb_$v.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/va_pb_$v.json').read().strip().splitlines()[-1]); print('vanilla per-batch v22=$v', r['value'], r['ms_per_step'])" | tee -a $O/bench_ab.txt
done
for v in -1 2 4 -1 2 4; do
  echo "variant 22=$v" >> $O/wgbench_tp.txt
  timeout -k 10 200 python scripts/wgbench.py --iters 50 --variant 22=$v >> $O/wgbench_tp.txt 2>&1 || { echo WGB_FAIL; tail $O/wgbench_tp.txt; exit 1; }
done
grep -E "variant|group" $O/wgbench_tp.txt
