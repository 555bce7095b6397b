#!/bin/bash
# round 6: the U-shape persistent epoch -- tests, then the U-shape bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_us
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_ushape_persist_gpu.py "tests/test_golden_modes_gpu.py::test_ushape_split_epoch_matches_composed_torch_adam_every_step" "tests/test_golden_modes_gpu.py::test_ushape_lookahead_epoch_free_running_matches_torch" > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" $O/tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode ushape --steps 20 --warmup 5 --json_out $O/bench_ushape.json > $O/bench_ushape.log 2>&1 || { echo "bench rc $?"; exit 1; }
python -c "import json; r=json.load(open('$O/bench_ushape.json')); print(r['value'], r['ms_per_step'], r['config'].get('split_epochs'), r['config'].get('split_persist_fallback'))"
