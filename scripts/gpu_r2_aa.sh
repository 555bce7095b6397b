#!/bin/bash
# Skinny forward: waves per workgroup (variant 14: 0 = 8, 3 = 4, 4 = 16; 2 = the k-loop form).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python scripts/native_ab.py --tp 1 2 4 8 --variants 14=0 14=3 14=4 14=2 --rounds 3 --epochs 3 > gpurun_out/r2aa_native_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r2aa_native_ab.txt; exit 1; }
grep "us/step" gpurun_out/r2aa_native_ab.txt
