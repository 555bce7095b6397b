#!/bin/bash
# U-shape: kernel time per batch vs wall time (is the Python-issued split epoch host-bound?).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r2ab_prof" -o u -- python3 "$R/bench.py" --mode ushape --steps 1 --warmup 0 --num_samples 20000 --json_out "$R/gpurun_out/r2ab_ushape.json" > "$R/gpurun_out/r2ab_prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/r2ab_prof.log"; exit 1; }
echo PROF_OK
