#!/bin/bash
# One GPU-box iteration (round 4): selected GPU tests, then optional bench / profile.
#   TESTS="tests/test_x.py -k y" BENCH=1 PROF=1 bash scripts/gpu_r4.sh
# Outputs under gpurun_out/r4/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TMO:-900} python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r4/tests.log 2>&1 || { echo TEST_FAIL; grep -E "PASS|FAIL|Error|assert" gpurun_out/r4/tests.log | tail -40; tail -30 gpurun_out/r4/tests.log; exit 1; }
  grep -cE "PASSED" gpurun_out/r4/tests.log; tail -2 gpurun_out/r4/tests.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/r4/bench.log 2>&1 \
    || { echo BENCH_FAIL; tail -30 gpurun_out/r4/bench.log; exit 1; }
  tail -1 gpurun_out/r4/bench.log
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r4/prof" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 > "$R/gpurun_out/r4/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/r4/prof.log"; exit 1; }
  echo prof-done
fi
