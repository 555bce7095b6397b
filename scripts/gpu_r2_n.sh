#!/bin/bash
# Validation after the one-round-trip forward default and the split-mode order policy:
# every GPU test, smoke, the N=1 headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2n_tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAILED|^E " gpurun_out/r2n_tests.log | head -20; tail -5 gpurun_out/r2n_tests.log; exit 1; }
tail -1 gpurun_out/r2n_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2n_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r2n_smoke.log; exit 1; }
tail -1 gpurun_out/r2n_smoke.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --json_out gpurun_out/r2n_bench_n1.json > gpurun_out/r2n_bench_n1.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r2n_bench_n1.log; exit 1; }
tail -1 gpurun_out/r2n_bench_n1.log | cut -c1-220
timeout -k 10 300 ./scripts/probe/dgrad_probe > gpurun_out/r2n_dgrad_probe.txt 2>&1 || { echo DPROBE_FAIL; tail gpurun_out/r2n_dgrad_probe.txt; exit 1; }
echo DPROBE_OK
