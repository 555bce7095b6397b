#!/bin/bash
# round 6: U-shape persistent epoch incl. its bf16 instantiation -- tests, then fp32 / bf16 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_usbf
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ushape_persist_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASSED|FAILED|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -12
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --mode ushape --dtype $dt --steps 20 --warmup 5 --json_out $O/bench_us_$dt.json > $O/bench_us_$dt.log 2>&1 || { echo "bench $dt rc $?"; tail $O/bench_us_$dt.log; exit 1; }
  python -c "import json; r=json.load(open('$O/bench_us_$dt.json')); print('$dt', r['value'], r['ms_per_step'], r['dtype'], r['config'].get('split_epochs'), r['config'].get('split_persist_fallback'))"
done
