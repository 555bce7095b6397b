#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_drift
mkdir -p $O
timeout -k 10 300 python scripts/probe/synced_drift.py hybrid 1000 > $O/synced_hybrid.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/probe/synced_drift.py lps 1000 > $O/synced_lps.txt 2>&1 || exit 1
