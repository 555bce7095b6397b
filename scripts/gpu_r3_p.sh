#!/bin/bash
# Round 3, call P: rocprofv3 kernel tables of the U-shape bench in fp32 and bf16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof_$dt -o prof -- python3 bench.py --mode ushape --dtype $dt --steps 1 --warmup 1 > gpurun_out/r3p_$dt.log 2>&1 || { tail -20 gpurun_out/r3p_$dt.log; exit 1; }
  f=$(find gpurun_out/r3p_prof_$dt -name '*kernel_stats.csv' | sort | tail -1)
  cp "$f" gpurun_out/r3p_ushape_${dt}_kernel_stats.csv
  find gpurun_out/r3p_prof_$dt -name '*.csv' -delete
  echo "== $dt"; python scripts/kstats.py gpurun_out/r3p_ushape_${dt}_kernel_stats.csv | head -14
done
