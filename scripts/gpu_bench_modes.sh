#!/bin/bash
# GPU tests, then bench.py in every mode on one MI355X.  -> gpurun_out/bench_<mode>.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/t.log; exit 1; }
  tail -2 gpurun_out/t.log
fi
for m in ${MODES:-sisa vanilla ushape concat}; do
  timeout -k 10 300 python bench.py --mode $m --steps ${STEPS:-5} --warmup 2 --json_out gpurun_out/bench_$m.json > gpurun_out/bench_$m.log 2>&1 || { echo "BENCH_FAIL $m"; tail -30 gpurun_out/bench_$m.log; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/bench_$m.json'));print('$m', r['value'], r['ms_per_step'], r['vs_baseline'])"
done
