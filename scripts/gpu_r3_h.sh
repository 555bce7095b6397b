#!/bin/bash
# Round 3, call H: concat native-vs-Python bitwise test; rocprofv3 kernel tables of the native
# server step at TP = 1 and a TP = 8 shard (1-rank peer-mapped all-reduce stand-in).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_split_native_gpu.py > gpurun_out/r3h_tests.log 2>&1 || { tail -60 gpurun_out/r3h_tests.log; exit 1; }
tail -4 gpurun_out/r3h_tests.log
for tp in 1 8; do
  $T 300 python -u scripts/prof_step.py --path native --tp $tp --allreduce ipc --steps 640 --time > gpurun_out/r3h_step_tp$tp.txt 2>&1 || { tail -20 gpurun_out/r3h_step_tp$tp.txt; exit 1; }
  grep us_per_step gpurun_out/r3h_step_tp$tp.txt
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h_prof_tp$tp -o prof -- python3 scripts/prof_step.py --path native --tp $tp --allreduce ipc --steps 640 > gpurun_out/r3h_prof_tp$tp.log 2>&1 || { tail -20 gpurun_out/r3h_prof_tp$tp.log; exit 1; }
  f=$(find gpurun_out/r3h_prof_tp$tp -name '*kernel_stats.csv' | sort | tail -1)
  cp "$f" gpurun_out/r3h_tp${tp}_kernel_stats.csv
  find gpurun_out/r3h_prof_tp$tp -name '*.csv' -delete
  echo "== TP $tp"; python scripts/kstats.py gpurun_out/r3h_tp${tp}_kernel_stats.csv
done
