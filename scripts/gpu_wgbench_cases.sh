#!/bin/bash
# wgrad_group alone on the split modes' and concat's layers, per cache-policy preset (variant
# 21: 6 = the cache-resident form, 1 = the over-cache form).  -> gpurun_out/wgb.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out" && cd "$R"
for c in ushape vanilla concat; do
  for p in 6 1 4 5 6 1; do
    timeout -k 10 120 python -u scripts/wgbench.py --case $c --iters 50 --variant 21=$p 2>&1 | grep -v amdgpu >> gpurun_out/wgb.log || { echo WGB_FAIL $c $p; exit 1; }
  done
done
cat gpurun_out/wgb.log
