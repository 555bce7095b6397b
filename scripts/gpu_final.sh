#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), and the N=1 bench for every mode.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log
