#!/bin/bash
# round 6: vanilla forward-pass ring depth A/B (timing + bitwise equality across depths and
# repeats), then the long-launch, hybrid, vanilla-persist and resident T = 2 tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_ring
T=$(mktemp -d)
mkdir -p $O
for r in 1; do for v in ring4 ring2; do
  echo "== $v pass $r" >> $O/trace.log
  timeout -k 10 150 python -u ab/$v/scripts/vanilla_trace.py --reps 5 --batches 600 >> $O/trace.log 2>&1 || { echo "trace $v rc $?"; exit 1; }
done; done
for v in ring4 ring2 ring6; do
  timeout -k 10 120 python -u ab/$v/scripts/probe/va_state_dump.py $T/state_$v.pt 1000 >> $O/dump.log 2>&1 || { echo "dump $v rc $?"; exit 1; }
  timeout -k 10 120 python -u ab/$v/scripts/probe/va_state_dump.py $T/state2_$v.pt 1000 >> $O/dump.log 2>&1 || { echo "dump2 $v rc $?"; exit 1; }
done
python scripts/probe/va_state_cmp.py $T/state_ring2.pt $T/state2_ring2.pt $T/state_ring4.pt $T/state2_ring4.pt $T/state_ring6.pt $T/state2_ring6.pt > $O/cmp.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_long_launch_gpu.py tests/test_hybrid_gpu.py tests/test_vanilla_persist_gpu.py > $O/tests.log 2>&1
echo "tests rc $?"
