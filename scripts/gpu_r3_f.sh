#!/bin/bash
# Round 3, call F: streaming wgrad form (variant 12) — bitwise test, server-step A/B at every
# TP shard, wgrad microbenchmark, and the mode benches with it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/r3f_tests.log 2>&1 || { tail -60 gpurun_out/r3f_tests.log; exit 1; }
tail -4 gpurun_out/r3f_tests.log
$T 400 python -u scripts/native_ab.py --tp 1 2 4 8 --allreduce ipc --variants 12=0 12=1 > gpurun_out/r3f_native_ab.txt 2>&1 || { tail -30 gpurun_out/r3f_native_ab.txt; exit 1; }
cat gpurun_out/r3f_native_ab.txt
$T 200 python -u scripts/wgbench.py --tps 1 8 > gpurun_out/r3f_wgbench_v0.txt 2>&1 && $T 200 python -u scripts/wgbench.py --tps 1 8 --variant 12=1 > gpurun_out/r3f_wgbench_v1.txt 2>&1 || { tail -30 gpurun_out/r3f_wgbench_v*.txt; exit 1; }
tail -12 gpurun_out/r3f_wgbench_v0.txt gpurun_out/r3f_wgbench_v1.txt
for m in "sisa 2" "vanilla 2"; do
  set -- $m
  $T 300 python -u bench.py --mode $1 --world_size $2 --steps 2 --warmup 1 --kernel_variant 12=1 --json_out gpurun_out/r3f_bench_$1_v1.json > gpurun_out/r3f_bench_$1_v1.log 2>&1 || { tail -20 gpurun_out/r3f_bench_$1_v1.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3f_bench_$1_v1.json'));print('$1 v12=1', d['value'], d['config']['phase_seconds'])"
done
