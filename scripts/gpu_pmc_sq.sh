#!/bin/bash
# One SQ counter pass (LDS bank conflicts / LDS and VALU instruction counts) over the wgrad
# microbench at TP = 1 and 8.  -> gpurun_out/pmc_sq/, gpurun_out/pmc_sq_summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_sq" -o wg -- \
  python3 "$R/scripts/wgbench.py" --tps 1 8 --iters 10 > "$R/gpurun_out/pmc_sq.log" 2>&1 || { echo "PMC_FAIL"; tail -20 "$R/gpurun_out/pmc_sq.log"; exit 1; }
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out" > "$R/gpurun_out/pmc_sq_summary.txt" && grep -E "== |sl::" "$R/gpurun_out/pmc_sq_summary.txt"
