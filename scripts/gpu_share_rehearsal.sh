#!/bin/bash
# N > 1 rehearsal on a one-GPU box: bench.py's full SISA schedule with N ranks on cuda:0
# (gloo control + host-staged p2p, Bob TP = N with the peer-mapped all-reduce).  Not a
# scaling measurement: the ranks share one GPU's CUs and HBM.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for N in ${NS:-2 4}; do
  timeout -k 10 ${TMO:-300} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29700 + N)) bench.py --gpus $N --ranks_share_gpu --steps ${STEPS:-1} --warmup ${WARM:-1} \
    --json_out gpurun_out/share_n$N.json > gpurun_out/share_n$N.log 2>&1 || { echo "N=$N FAIL"; tail -40 gpurun_out/share_n$N.log; exit 1; }
  echo "N=$N ok: $(cut -c1-400 gpurun_out/share_n$N.json)"
done
