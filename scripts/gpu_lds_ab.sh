#!/bin/bash
# Look-ahead LDS padding (variant 1): GPU tests, SQ LDS counter pass, native-executor A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lds.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t_lds.log; exit 1; }
tail -1 gpurun_out/t_lds.log
bash scripts/gpu_pmc_sq.sh || exit 1
cd "$R"
timeout -k 10 400 python -u scripts/native_ab.py --tp 1 2 8 --variants 1=0 1=1 1=0,6=0 > gpurun_out/native_ab_lds.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/native_ab_lds.txt; exit 1; }
grep "^tp=" gpurun_out/native_ab_lds.txt
