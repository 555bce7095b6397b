#!/bin/bash
# Wgrad traversal / store-form A/B on one MI355X: kernel tests, then scripts/cache_ab.py
# at TP shard sizes 1 2 4 8 and the wgrad microbench per variant.  -> gpurun_out/cache_ab.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad_group" > gpurun_out/t_wg.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t_wg.log; exit 1; }
tail -1 gpurun_out/t_wg.log
timeout -k 10 400 python -u scripts/cache_ab.py --tp 1 2 4 8 ${AB_ARGS} > gpurun_out/cache_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/cache_ab.txt; exit 1; }
cat gpurun_out/cache_ab.txt
for v in ${WGB_VARIANTS:-"7=1" "7=0" "4=1"}; do
  echo "== wgbench variant $v" >> gpurun_out/cache_ab.txt
  timeout -k 10 200 python -u scripts/wgbench.py --iters 100 --variant $v >> gpurun_out/cache_ab.txt 2>&1 || { echo WGB_FAIL; exit 1; }
done
tail -20 gpurun_out/cache_ab.txt
