#!/bin/bash
# Round 3, call V: the fp32 GEMM tile forms (BK 16 vs 32) on the evaluation shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gemm_bench.py --forms 0 2 --shapes all --reps 16 > gpurun_out/r3v_gemm_forms.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r3v_gemm_forms.txt
exit $rc
