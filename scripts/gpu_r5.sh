#!/bin/bash
# One GPU-box iteration (round 5): selected GPU tests, then optional bench / profile.
#   TESTS="tests/test_x.py -k y" BENCH=1 PROF=1 bash scripts/gpu_r5.sh
# Outputs under gpurun_out/$OUT/ (OUT defaults to r5).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r5}
cd "$R" && mkdir -p gpurun_out/$OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TMO:-900} python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/$OUT/tests.log 2>&1 || { echo TEST_FAIL; grep -E "PASS|FAIL|Error|assert" gpurun_out/$OUT/tests.log | tail -40; tail -30 gpurun_out/$OUT/tests.log; exit 1; }
  grep -cE "PASSED" gpurun_out/$OUT/tests.log; tail -2 gpurun_out/$OUT/tests.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/$OUT/bench.log 2>&1 \
    || { echo BENCH_FAIL; tail -30 gpurun_out/$OUT/bench.log; exit 1; }
  tail -1 gpurun_out/$OUT/bench.log
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$OUT/prof" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 > "$R/gpurun_out/$OUT/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/$OUT/prof.log"; exit 1; }
  echo prof-done
fi
