#!/bin/bash
# Every mode's full schedule at ws = 2 / 3 / 5 / 9 on one MI355X (co-located Alices): bench.py JSON lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r2_modes
export TMPDIR=/tmp
for mode in sisa concat control vanilla ushape; do
  for ws in 2 3 5 9; do
    timeout -k 10 300 python bench.py --mode $mode --world_size $ws --steps 2 --warmup 1 --json_out gpurun_out/r2_modes/${mode}_ws$ws.json > gpurun_out/r2_modes/${mode}_ws$ws.log 2>&1 || { echo FAIL $mode $ws; tail -5 gpurun_out/r2_modes/${mode}_ws$ws.log; exit 1; }
    echo "$mode ws=$ws $(python -c "import json;d=json.load(open('gpurun_out/r2_modes/${mode}_ws$ws.json'));print(d['value'], d['ms_per_step'])")"
  done
done
