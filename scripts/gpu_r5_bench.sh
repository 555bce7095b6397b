#!/bin/bash
# Round-5 tests + benches: GPU tests named by TESTS, then the N = 1 headline bench and the
# ws = 9 SISA / concat points on one GPU.  Outputs: gpurun_out/$OUT/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r5b2}
cd "$R" && mkdir -p gpurun_out/$OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/$OUT/tests.log | tail -20; tail -3 gpurun_out/$OUT/tests.log; exit 1; }
  tail -1 gpurun_out/$OUT/tests.log
fi
for spec in ${BENCHES:-"n1:--steps 3 --warmup 1" "ws9:--world_size 9 --steps 2 --warmup 1"}; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python bench.py $args > gpurun_out/$OUT/bench_$name.json 2> gpurun_out/$OUT/bench_$name.err || { echo BENCH_FAIL $name; tail -20 gpurun_out/$OUT/bench_$name.err; exit 1; }
  python - "$name" gpurun_out/$OUT/bench_$name.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1], d["value"], d["ms_per_step"], c.get("server_executor"), c.get("server_executor_reason"), c.get("server_executor_fallback"), c.get("phase_seconds"))
PY
done
