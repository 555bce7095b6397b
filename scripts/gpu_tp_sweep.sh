#!/bin/bash
# Wall-clock us/step of Bob's server step at every TP shard size (1-rank communicator,
# so the all-reduce cost of a real multi-GPU run is NOT included).  -> gpurun_out/tp_sweep.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/tp_sweep.txt
for tp in ${TPS:-1 2 4 8}; do
  for p in ${PATHS:-lookahead graph}; do
    timeout -k 10 120 python scripts/prof_step.py --path $p --tp $tp --steps ${STEPS:-640} --time $EXTRA >> gpurun_out/tp_sweep.txt 2>&1 || { echo "SWEEP_FAIL $p $tp"; tail -20 gpurun_out/tp_sweep.txt; exit 1; }
  done
done
cat gpurun_out/tp_sweep.txt
