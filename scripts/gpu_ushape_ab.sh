#!/bin/bash
# bench.py A/B of kernel variant 1 (look-ahead LDS tile padding; 1=1 = unpadded rows) per mode,
# interleaved runs on one box.  MODES="ushape vanilla sisa" by default.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out
for m in ${MODES:-ushape vanilla sisa}; do
  for i in 1 2; do
    for v in "" "--kernel_variant 1=1"; do
      timeout -k 10 200 python bench.py --mode $m --steps 5 --warmup 2 $v > gpurun_out/ab_$m.log 2>&1 || { tail -20 gpurun_out/ab_$m.log; exit 1; }
      python -c "import json;r=json.loads(open('gpurun_out/ab_$m.log').read().strip().splitlines()[-1]);print('$m','${v:-default}',r['value'],r['ms_per_step'])"
    done
  done
done
