#!/bin/bash
# DPP wave / lane-group reductions everywhere + the DPP head: all GPU tests, smoke, benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2r_tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAILED|^E " gpurun_out/r2r_tests.log | head -20; tail -5 gpurun_out/r2r_tests.log; exit 1; }
tail -1 gpurun_out/r2r_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2r_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r2r_smoke.log; exit 1; }
tail -1 gpurun_out/r2r_smoke.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --json_out gpurun_out/r2r_bench_n1.json > gpurun_out/r2r_bench_n1.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r2r_bench_n1.log; exit 1; }
tail -1 gpurun_out/r2r_bench_n1.log | cut -c1-200
for mode in ushape vanilla; do
  timeout -k 10 300 python bench.py --mode $mode --steps 3 --warmup 1 --json_out gpurun_out/r2r_$mode.json > gpurun_out/r2r_$mode.log 2>&1 || { echo MODE_FAIL $mode; tail -20 gpurun_out/r2r_$mode.log; exit 1; }
  tail -1 gpurun_out/r2r_$mode.log | cut -c1-200
done
timeout -k 10 300 python scripts/native_ab.py --tp 1 2 4 8 --variants 0=0 --rounds 3 --epochs 3 > gpurun_out/r2r_native_steps.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2r_native_steps.txt; exit 1; }
grep "us/step" gpurun_out/r2r_native_steps.txt
