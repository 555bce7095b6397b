#!/bin/bash
# Round 3, call C: whole GPU suite on the cleaned-up tree, then the headline bench and every
# mode's schedule (concat ws = 9 for the eval cost).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r3c_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r3c_gpu_suite.log
$T 400 python -u bench.py --steps 5 --warmup 2 --json_out gpurun_out/r3c_bench_n1.json > gpurun_out/r3c_bench_n1.log 2>&1 || { tail -20 gpurun_out/r3c_bench_n1.log; exit 1; }
cat gpurun_out/r3c_bench_n1.json
for m in "concat 9" "vanilla 2" "ushape 2" "sisa 9"; do
  set -- $m
  $T 300 python -u bench.py --mode $1 --world_size $2 --steps 2 --warmup 1 --json_out gpurun_out/r3c_bench_$1_ws$2.json > gpurun_out/r3c_bench_$1_ws$2.log 2>&1 || { tail -20 gpurun_out/r3c_bench_$1_ws$2.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3c_bench_$1_ws$2.json'));print('$1 ws$2', d['value'], d['config']['phase_seconds'])"
done
