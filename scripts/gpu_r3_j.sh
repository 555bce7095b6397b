#!/bin/bash
# Round 3, call J: GEMM numerics + forms vs hipBLASLt (call I), then the default N = 1 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash scripts/gpu_r3_i.sh || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || { tail -20 gpurun_out/r3j_bench.err; exit 1; }
cat gpurun_out/r3j_bench.json
