#!/bin/bash
# Round-5 vanilla persistent epoch: its GPU tests (TESTS), then vanilla ws = 2 benches with the
# persistent executor and without it (--split_persist off), and optionally the headline bench.
# Outputs: gpurun_out/$OUT/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r5x_va}
cd "$R" && mkdir -p gpurun_out/$OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/$OUT/tests.log | tail -30; tail -5 gpurun_out/$OUT/tests.log; exit 1; }
  tail -1 gpurun_out/$OUT/tests.log
fi
bench() {
  name=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/$OUT/bench_$name.json 2> gpurun_out/$OUT/bench_$name.err || { echo BENCH_FAIL $name; tail -20 gpurun_out/$OUT/bench_$name.err; return 1; }
  python - "$name" gpurun_out/$OUT/bench_$name.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1], d["value"], d["ms_per_step"], c.get("split_epochs"), c.get("split_persist_fallback"),
      c.get("server_executor"), c.get("phase_seconds"))
PY
}
if [ -z "$NOBENCH" ]; then
  bench va --mode vanilla --steps ${STEPS:-2} --warmup 1 &&
  bench vaoff --mode vanilla --split_persist off --steps ${STEPS:-2} --warmup 1 || exit 1
fi
if [ -n "$HEADLINE" ]; then
  bench n1 --steps 3 --warmup 1 || exit 1
fi
