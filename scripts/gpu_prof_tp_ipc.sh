#!/bin/bash
# Kernel table of a TP shard's native server step with the fused peer-mapped all-reduce
# (1-rank stand-in), TP = 8 and TP = 2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
for T in 8 2; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_tp$T" -o st -- \
     python3 "$R/scripts/native_ab.py" --tp $T --variants 0=0 --rounds 1 --epochs 3 --allreduce ipc) \
     > gpurun_out/prof_tp$T.log 2>&1 || { echo "prof tp=$T FAIL"; tail -20 gpurun_out/prof_tp$T.log; exit 1; }
  f=$(find gpurun_out/prof_tp$T -name '*kernel_stats.csv' | head -1)
  echo "== TP=$T ($f)"; python3 scripts/kstats.py "$f"
done
