#!/bin/bash
# Round-5 hybrid iteration: the persistent-epoch GPU tests, the per-seam critical-path trace at
# TP = 1 / 2 / 4 against launch-per-stage, and a short N = 1 bench.  Outputs: gpurun_out/$OUT/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r5h}
cd "$R" && mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_hybrid_gpu.py tests/test_resident_gpu.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/$OUT/tests.log | tail -30; tail -5 gpurun_out/$OUT/tests.log; exit 1; }
tail -1 gpurun_out/$OUT/tests.log
timeout -k 10 400 python -u scripts/hybrid_ab.py --tp ${TPS:-1 2 4} --steps 500 --rounds 3 --trace > gpurun_out/$OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -30 gpurun_out/$OUT/trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$OUT/trace.log | grep -v "trace wg"
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/$OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/$OUT/bench.log; exit 1; }
  tail -1 gpurun_out/$OUT/bench.log | cut -c1-300
fi
