#!/bin/bash
# Kernel tables of the native server step at a TP = 8 shard and at TP = 1 (rocprofv3 kernel trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for tp in 8 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r2x_tp$tp" -o k -- python3 "$R/scripts/native_ab.py" --tp $tp --variants 0=0 --rounds 1 --epochs 2 > "$R/gpurun_out/r2x_tp$tp.log" 2>&1 || { echo PROF_FAIL $tp; tail -20 "$R/gpurun_out/r2x_tp$tp.log"; exit 1; }
  echo PROF_OK $tp
done
