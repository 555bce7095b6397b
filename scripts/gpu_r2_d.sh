#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python scripts/golden_diag.py > gpurun_out/r2d_golden_diag.txt 2>&1 || { echo DIAG_FAIL; tail -20 gpurun_out/r2d_golden_diag.txt; exit 1; }
cat gpurun_out/r2d_golden_diag.txt
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_emulation_gpu.py -v --timeout 200 --timeout-method thread -k "multi_alice or tp_emul or dgrad" > gpurun_out/r2d_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|^E " gpurun_out/r2d_tests.log | head -30; tail -2 gpurun_out/r2d_tests.log
[ $rc -le 1 ] || exit $rc
for v in serial multi; do
  extra=""; [ $v = serial ] && extra="--serial_alices"
  timeout -k 10 300 python -c "
import sys, bench
" > /dev/null 2>&1
done
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --world_size 9 --server_epochs 1 > gpurun_out/r2d_ws9_multi.json 2>&1 || { echo B1_FAIL; tail -5 gpurun_out/r2d_ws9_multi.json; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2d_ws9_multi.json').read().strip().splitlines()[-1]);print('multi', d['config']['phase_seconds'])"
