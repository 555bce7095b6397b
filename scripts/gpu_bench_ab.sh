#!/bin/bash
# bench.py A/B of kernel variants, interleaved: for each mode, REPS rounds of (default, each
# VARIANT).  -> gpurun_out/bench_ab.txt    e.g. MODES="ushape" VARIANTS="4=1 7=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/bench_ab.txt
for m in ${MODES:-ushape}; do
  for rep in $(seq ${REPS:-2}); do
    for v in default ${VARIANTS:-4=1}; do
      va=""; [ "$v" != default ] && va="--kernel_variant $v"
      timeout -k 10 300 python bench.py --mode $m --steps ${STEPS:-5} --warmup 2 $va > gpurun_out/ab_run.log 2>&1 || { echo "BENCH_FAIL $m $v"; tail -20 gpurun_out/ab_run.log; exit 1; }
      python -c "import json,sys;r=json.loads(open('gpurun_out/ab_run.log').read().strip().splitlines()[-1]);print('$m', '$v', r['value'], r['ms_per_step'])" >> gpurun_out/bench_ab.txt
    done
  done
done
cat gpurun_out/bench_ab.txt
