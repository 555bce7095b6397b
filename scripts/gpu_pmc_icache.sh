#!/bin/bash
# Instruction-cache counters of the hybrid persistent epoch at TP = 1 (the phase code of the
# head chain runs once per step between streams of 325 MB): SQC instruction-cache requests /
# hits / misses and the SQ's instruction-fetch waits, one counter group per run, plain launches
# of 256 workgroups.  -> gpurun_out/pmci/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pmci"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  SL_PERSIST_WORKGROUPS=256 timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/p$i" -o hy -- \
    python3 "$R/scripts/hybrid_ab.py" --tp 1 --steps 200 --rounds 1 --only hybrid > "$O/p$i.log" 2>&1 || { echo "PMC_FAIL $c"; tail -20 "$O/p$i.log"; exit 1; }
done
echo done
