#!/bin/bash
# Round 2 refresh: every GPU test, smoke, the N=1 headline bench, co-located ws=5/9 runs of sisa and
# concat, and a kernel-trace profile of one full-schedule step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2i_tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAILED|^E " gpurun_out/r2i_tests.log | head -20; tail -5 gpurun_out/r2i_tests.log; exit 1; }
tail -1 gpurun_out/r2i_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2i_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r2i_smoke.log; exit 1; }
tail -1 gpurun_out/r2i_smoke.log
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --json_out gpurun_out/r2i_bench_n1.json > gpurun_out/r2i_bench_n1.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r2i_bench_n1.log; exit 1; }
tail -1 gpurun_out/r2i_bench_n1.log | cut -c1-200
for mode in sisa concat; do
  for ws in 5 9; do
    timeout -k 10 300 python bench.py --mode $mode --world_size $ws --steps 1 --warmup 1 --json_out gpurun_out/r2i_${mode}_ws$ws.json > gpurun_out/r2i_${mode}_ws$ws.log 2>&1 || { echo WS_FAIL $mode $ws; tail -20 gpurun_out/r2i_${mode}_ws$ws.log; exit 1; }
    tail -1 gpurun_out/r2i_${mode}_ws$ws.log | cut -c1-200
  done
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r2i_prof" -o r2i -- python "$R/bench.py" --steps 1 --warmup 0 --server_epochs 1 > "$R/gpurun_out/r2i_prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/r2i_prof.log"; exit 1; }
echo PROF_OK
