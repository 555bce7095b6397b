#!/bin/bash
# round 6: vanilla forward pass with W loaded straight in the MFMA B layout (direct) against the
# LDS-staged form (staged): timing (trace, interleaved), 1,000-step states bitwise across the two,
# the vanilla tests, then the ws = 2 vanilla bench (direct)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_vafwd
T=$(mktemp -d)
mkdir -p $O
for r in 1 2; do for v in direct staged; do
  echo "== $v pass $r" >> $O/trace.log
  timeout -k 10 150 python -u ab/$v/scripts/vanilla_trace.py --reps 5 --batches 600 >> $O/trace.log 2>&1 || { echo "trace $v rc $?"; exit 1; }
done; done
grep -E "==|us/step|fwd done|x rel" $O/trace.log
for v in direct staged; do
  timeout -k 10 120 python -u ab/$v/scripts/probe/va_state_dump.py $T/state_$v.pt 1000 >> $O/dump.log 2>&1 || { echo "dump $v rc $?"; exit 1; }
done
timeout -k 10 120 python -u ab/direct/scripts/probe/va_state_dump.py $T/state2_direct.pt 1000 >> $O/dump.log 2>&1 || { echo "dump2 rc $?"; exit 1; }
python scripts/probe/va_state_cmp.py $T/state_staged.pt $T/state_direct.pt $T/state2_direct.pt | tee $O/cmp.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vanilla_persist_gpu.py tests/test_long_launch_gpu.py::test_vanilla_epoch_long_launch tests/test_golden_gpu.py::test_vanilla_split_epoch_matches_composed_torch_sgd > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASSED|FAILED|Error" $O/tests.log | tail; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode vanilla --steps 20 --warmup 5 > $O/bench_va_$i.json 2> $O/bench_va_$i.err || { echo VBENCH_FAIL; tail $O/bench_va_$i.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/bench_va_$i.json').read().strip().splitlines()[-1]); print('vanilla', r['value'], r['ms_per_step'], r['config'].get('split_epochs'), r['config'].get('split_persist_fallback'))"
done
