#!/bin/bash
# Hardware-counter passes (one counter group per run) over the wgrad+optimizer microbench at
# TP = 1 and 8: bytes fetched from / written to memory past L2 per kernel dispatch.
# -> gpurun_out/pmc_{fetch,write}/ and gpurun_out/pmc_summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$c" -o wg -- \
    python3 "$R/scripts/wgbench.py" --tps 1 8 --iters 20 > "$R/gpurun_out/pmc_$c.log" 2>&1 || { echo "PMC_FAIL $c"; tail -20 "$R/gpurun_out/pmc_$c.log"; exit 1; }
done
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out" > "$R/gpurun_out/pmc_summary.txt" && cat "$R/gpurun_out/pmc_summary.txt"
