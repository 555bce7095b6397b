#!/bin/bash
# Round 3, call N: resident-epoch tests (incl. the SISA session path and two processes on one
# GPU), the A/B, and a rocprofv3 kernel table of both executors at a TP = 8 shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resident_gpu.py > gpurun_out/r3n_tests.log 2>&1
rc=$?
tail -14 gpurun_out/r3n_tests.log
[ $rc -eq 0 ] || { tail -80 gpurun_out/r3n_tests.log; exit 1; }
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n_prof -o prof -- python3 scripts/resident_ab.py --tp 8 --steps 437 --rounds 2 --epochs 2 > gpurun_out/r3n_prof.log 2>&1 || { tail -20 gpurun_out/r3n_prof.log; exit 1; }
f=$(find gpurun_out/r3n_prof -name '*kernel_stats.csv' | sort | tail -1)
cp "$f" gpurun_out/r3n_tp8_kernel_stats.csv
find gpurun_out/r3n_prof -name '*.csv' -delete
python scripts/kstats.py gpurun_out/r3n_tp8_kernel_stats.csv
grep "us/step" gpurun_out/r3n_prof.log
