#!/bin/bash
# Round 3, call W: first-chunk A / dZ loads ahead of W / m / v in the wgrad launch (variant 6 = 1) against
# the state-first order, per server step at TP 1 / 4 / 8 shard shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/native_ab.py --tp 1 4 8 --variants 6=0 6=1 --allreduce ipc --rounds 5 --epochs 3 > gpurun_out/r3w_afirst_ab.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r3w_afirst_ab.txt
exit $rc
