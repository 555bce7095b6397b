#!/bin/bash
# round 6: hand-off stress test; reproduce the resident T = 2 two-process anomaly
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_diag
mkdir -p $O
timeout -k 10 240 python scripts/handoff_stress.py 2000 > $O/handoff_stress.txt 2>&1 || { echo "stress rc $?"; exit 1; }
timeout -k 10 150 python scripts/diag_persist_tp.py resident 2 6 > $O/diag_res_2eng.txt 2>&1 || { echo "diag1 rc $?"; exit 1; }
ALT=1 timeout -k 10 150 python scripts/diag_persist_tp.py resident 2 6 > $O/diag_res_2eng_alt.txt 2>&1 || { echo "diag2 rc $?"; exit 1; }
for k in 1 2 3; do
  timeout -k 10 150 python scripts/persist_fallback_one_gpu.py 2 resident > $O/fallback_res_$k.txt 2>&1
  rc=$?
  echo "fallback resident run $k rc $rc"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
