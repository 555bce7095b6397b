#!/bin/bash
# round 6: vanilla update runs dealt to XCDs by row band (SL_VA_XCD_RUNS=1, the default) against
# dealt in order (=0): the vanilla GPU tests, then interleaved vanilla_trace passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_xcdruns
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_vanilla_persist_gpu.py tests/test_split_remote_gpu.py tests/test_long_launch_gpu.py tests/test_golden_gpu.py tests/test_split_native_gpu.py -m gpu > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -20 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/tests.log
for r in $(seq ${PASSES:-3}); do
  for v in 1 0; do
    echo "== xcd_runs=$v" >> $O/ab.log
    SL_VA_XCD_RUNS=$v timeout -k 10 150 python -u scripts/vanilla_trace.py --batches 400 --reps 5 >> $O/ab.log 2>&1 || { echo TRACE_FAIL; exit 1; }
  done
done
