#!/bin/bash
# Round 3, call M: register-resident epoch (8-wave workgroups, no spills) — tests, timeline, A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resident_gpu.py > gpurun_out/r3m_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3m_tests.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/r3m_tests.log; exit 1; }
$T 200 python -u scripts/resident_trace.py --tp 8 > gpurun_out/r3m_trace.txt 2>&1 || { tail -30 gpurun_out/r3m_trace.txt; exit 1; }
cat gpurun_out/r3m_trace.txt
$T 300 python -u scripts/resident_ab.py --tp 8 --steps 437 --rounds 5 > gpurun_out/r3m_ab.txt 2>&1 || { tail -30 gpurun_out/r3m_ab.txt; exit 1; }
cat gpurun_out/r3m_ab.txt
