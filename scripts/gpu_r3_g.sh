#!/bin/bash
# Round 3, call G: vanilla fc2/fc3 update overlapped with the Alice's step (side stream) —
# bitwise tests against the Python loop, and the vanilla ws = 2 bench with / without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_split_native_gpu.py tests/test_kernels_gpu.py -k "split or wgrad" > gpurun_out/r3g_tests.log 2>&1 || { tail -60 gpurun_out/r3g_tests.log; exit 1; }
tail -4 gpurun_out/r3g_tests.log
for ov in 1 0 1 0; do
  SL_SPLIT_OVERLAP=$ov $T 300 python -u bench.py --mode vanilla --world_size 2 --steps 2 --warmup 1 --json_out gpurun_out/r3g_bench_vanilla_ov$ov.json > gpurun_out/r3g_bench_vanilla_ov$ov.log 2>&1 || { tail -20 gpurun_out/r3g_bench_vanilla_ov$ov.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3g_bench_vanilla_ov$ov.json'));print('vanilla overlap=$ov', d['value'], d['config']['phase_seconds'])"
done
