#!/bin/bash
# GPU tests, then the per-TP step-time sweep (scripts/gpu_tp_sweep.sh), then the N=1 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash scripts/gpu_tp_sweep.sh > /dev/null || exit 1
grep path= gpurun_out/tp_sweep.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
