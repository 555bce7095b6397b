#!/bin/bash
# Hardware counters of the vanilla persistent epoch (csrc/vanilla.hip, the direct-load forward
# pass): bytes fetched from / written past L2 and the L2 hit rate per launch of --batches steps,
# one counter group per run, plain launches of 256 workgroups (SL_PERSIST_WORKGROUPS=256).
# -> gpurun_out/pmcv/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pmcv"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $c | tr ' ' '_')
  SL_PERSIST_WORKGROUPS=256 timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/pmc_${tag}" -o va -- \
    python3 "$R/scripts/vanilla_trace.py" --reps 1 --batches 200 > "$O/pmc_${tag}.log" 2>&1 || { echo "PMC_FAIL $c"; tail -20 "$O/pmc_${tag}.log"; exit 1; }
done
python3 "$R/scripts/pmc_summary.py" "$O" > "$O/summary.txt" && grep -E "vanilla|==" "$O/summary.txt"
