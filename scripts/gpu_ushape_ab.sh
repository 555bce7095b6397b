#!/bin/bash
# U-shape fused middle + head (csrc/ushape.hip): the bitwise / golden tests, then the ws = 2
# U-shape bench interleaved fused / three-launch (variant 20 = 1).  -> gpurun_out/ush/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/ush"
mkdir -p "$O" && cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_split_native_gpu.py tests/test_golden_modes_gpu.py tests/test_kernels_gpu.py -k "ushape or head or split" -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" "$O/tests.log" | tail -20; tail -3 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python bench.py --mode ushape --steps 3 --warmup 1 --kernel_variant 20=$v > "$O/bench_v${v}_$r.json" 2> "$O/bench_v${v}_$r.err" || { echo BENCH_FAIL $v; tail -20 "$O/bench_v${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('variant20=$v', d['value'], d['ms_per_step'], d['config'].get('phase_seconds'))" "$O/bench_v${v}_$r.json"
  done
done
