#!/bin/bash
# Round 3, call L: phase timeline of the register-resident epoch at a TP = 8 shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/resident_trace.py --tp 8 > gpurun_out/r3l_trace.txt 2>&1 || { tail -30 gpurun_out/r3l_trace.txt; exit 1; }
cat gpurun_out/r3l_trace.txt
