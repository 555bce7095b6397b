#!/bin/bash
# Round 3, call T: rocprofv3 kernel table of the TP = 4 shard's server step (six-kernel chain,
# 1-rank peer-mapped stand-in).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3t_prof -o prof -- python3 $R/scripts/native_ab.py --tp 4 --variants chain=0 --allreduce ipc --rounds 1 --epochs 4 > $R/gpurun_out/r3t_prof.log 2>&1 || { tail -20 $R/gpurun_out/r3t_prof.log; exit 1; }
cd $R
f=$(find gpurun_out/r3t_prof -name '*kernel_stats.csv' | sort | tail -1)
cp "$f" gpurun_out/r3t_tp4_kernel_stats.csv
find gpurun_out/r3t_prof -name '*.csv' -delete
python scripts/kstats.py gpurun_out/r3t_tp4_kernel_stats.csv | head -20
grep "tp=4" gpurun_out/r3t_prof.log
