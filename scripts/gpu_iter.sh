#!/bin/bash
# One build->measure iteration on the GPU box: GPU tests, rocprofv3 kernel stats of the
# server-step variants, kernel microbench and the N=1 bench.  Outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TESTS=${TESTS:-tests -m gpu}
timeout -k 10 600 python -m pytest $TESTS -x -q > gpurun_out/t.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
PROF_PATHS=${PROF_PATHS:-"lookahead graph"} bash scripts/gpu_prof.sh || exit 1
timeout -k 10 400 python scripts/kbench.py --rounds 2 --iters 50 > gpurun_out/kbench.log 2>&1 || { echo KB_FAIL; tail -30 gpurun_out/kbench.log; exit 1; }
grep -E "bob_|fused:|v3:" gpurun_out/kbench.log | tail -24
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
