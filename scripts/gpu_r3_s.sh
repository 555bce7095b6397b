#!/bin/bash
# Round 3, call S: the chain launch against the six kernels per server step (TP 1..8 shard
# shapes, 1-rank peer-mapped stand-in), with the last chain launch's phase stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u scripts/native_ab.py --tp 1 2 4 8 --variants chain=0 chain=1 --allreduce ipc --rounds 3 --epochs 2 --trace > gpurun_out/r3s_chain_ab.txt 2>&1
rc=$?
cat gpurun_out/r3s_chain_ab.txt | grep -v amdgpu.ids
exit $rc
