#!/bin/bash
# Round 2, first call: GPU tests, smoke, the new full-schedule N=1 bench, and a kernel profile of it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2a_tests.log; exit 1; }
tail -2 gpurun_out/r2a_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r2a_smoke.log; exit 1; }
tail -1 gpurun_out/r2a_smoke.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/r2a_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r2a_bench.log; exit 1; }
tail -1 gpurun_out/r2a_bench.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --world_size 9 > gpurun_out/r2a_bench_ws9.log 2>&1 || { echo BENCH9_FAIL; tail -30 gpurun_out/r2a_bench_ws9.log; exit 1; }
tail -1 gpurun_out/r2a_bench_ws9.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r2a_prof" -o r2a -- python "$R/bench.py" --steps 1 --warmup 0 --server_epochs 1 > "$R/gpurun_out/r2a_prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/r2a_prof.log"; exit 1; }
echo PROF_OK
