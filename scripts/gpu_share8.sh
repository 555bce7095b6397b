#!/bin/bash
# One-GPU rehearsal of the driver's N = 8 launch: 8 ranks under torch.distributed.run, every rank
# on cuda:0 (--ranks_share_gpu: gloo control, host-staged data plane, Bob TP = 8 over the
# peer-mapped all-reduce, each persistent launch 32 workgroups).  Not a scaling measurement.
# -> gpurun_out/share8/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/share8"
mkdir -p "$O" && cd "$R"
for mode in ${MODES:-sisa}; do
  timeout -k 10 ${TMO:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29400 + RANDOM % 500)) bench.py --mode $mode --gpus 8 --steps 1 --warmup 0 --ranks_share_gpu \
    --num_samples ${NS:-18000} --json_out "$O/$mode.json" > "$O/$mode.log" 2>&1 || { echo "SHARE8_FAIL $mode"; tail -30 "$O/$mode.log"; exit 1; }
  python3 - "$O/$mode.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = d["config"]
print(c["mode"], d["value"], d["ms_per_step"], c["parallelism"], c["dist_world"], c.get("server_executor"),
      c.get("server_executor_reason"), c.get("server_executor_fallback"), c["phase_seconds"])
PY
done
