#!/bin/bash
# L2 hit rate of the fc2 forward / dgrad / head kernels with the XCD-grouped order (default)
# and the plain order (variant 19 = 2, 20 = 2): one rocprofv3 --pmc pass per order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
for V in "19=0,20=0" "19=2,20=2"; do
  tag=$(echo $V | tr ',=' '__')
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/pmc_xcd_$tag" -o p -- \
     python3 "$R/scripts/native_ab.py" --tp 1 --variants $V --rounds 1 --epochs 1) > gpurun_out/pmc_xcd_$tag.log 2>&1 \
     || { echo "pmc $V FAIL"; tail -20 gpurun_out/pmc_xcd_$tag.log; exit 1; }
  echo "pmc $V ok"
done
