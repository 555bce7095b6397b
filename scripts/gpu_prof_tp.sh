#!/bin/bash
# rocprofv3 kernel stats of Bob's look-ahead step at TP shard sizes (1-rank communicator).
# VARIANTS="1=1" passes kernel variants.  -> gpurun_out/prof_tp<T><tag>/ + a summary table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for tp in ${TPS:-1 8}; do
  for v in ${VARIANTS:-none}; do
    tag=""; va=""
    [ "$v" != none ] && { tag="_v${v/=/-}"; va="--variant $v"; }
    d="$R/gpurun_out/prof_tp${tp}${tag}"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o step -- \
      python3 "$R/scripts/prof_step.py" --path lookahead --steps 320 --tp $tp $va > "$d.log" 2>&1 || { echo "PROF_FAIL $tp $v"; tail -20 "$d.log"; exit 1; }
    echo "== tp=$tp variant=$v"
    python3 "$R/scripts/kstats.py" $(find "$d" -name "*kernel_stats.csv" | head -1)
  done
done
