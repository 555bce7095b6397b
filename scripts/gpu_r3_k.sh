#!/bin/bash
# Round 3, call K: register-resident server epoch — numerics tests, then step time against the
# launch-per-stage executor at a TP = 8 shard (1-rank peer-mapped stand-in).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resident_gpu.py > gpurun_out/r3k_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r3k_tests.log
[ $rc -eq 0 ] || exit 1
$T 300 python -u scripts/resident_ab.py --tp 8 --steps 437 --rounds 5 > gpurun_out/r3k_ab.txt 2>&1 || { tail -30 gpurun_out/r3k_ab.txt; exit 1; }
cat gpurun_out/r3k_ab.txt
