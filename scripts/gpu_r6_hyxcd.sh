#!/bin/bash
# round 6: hybrid stream runs dealt to XCDs by fc2 column block (SL_HY_XCD_RUNS=1, the default)
# against dealt in order (=0): the hybrid GPU tests, then interleaved hybrid_ab passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_hyxcd
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_hybrid_gpu.py tests/test_long_launch_gpu.py -m gpu > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -20 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/tests.log
for r in $(seq ${PASSES:-3}); do
  for v in 1 0; do
    echo "== hy_xcd_runs=$v" >> $O/ab.log
    SL_HY_XCD_RUNS=$v timeout -k 10 150 python -u scripts/hybrid_ab.py --tp 1 2 4 --steps 500 --rounds 3 --only hybrid >> $O/ab.log 2>&1 || { echo AB_FAIL; exit 1; }
  done
done
