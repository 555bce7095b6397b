#!/bin/bash
# Round-end rehearsal, as the driver runs it: every GPU test, smoke(), the N=1 bench at the
# driver's --steps 20 --warmup 5, then a kernel-trace profile of one full-schedule step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAILED|^E " gpurun_out/final_tests.log | head; tail -5 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
start=$(date +%s)
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --json_out gpurun_out/final_bench.json > gpurun_out/final_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/final_bench.log; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
tail -1 gpurun_out/final_bench.log | cut -c1-240
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final_prof" -o fp -- python "$R/bench.py" --steps 1 --warmup 0 > "$R/gpurun_out/final_prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/final_prof.log"; exit 1; }
echo PROF_OK
