#!/bin/bash
# fc2 dgrad split-N A/B on one MI355X: numerics of linear_dgrad at every variant-5 cap
# against torch, then scripts/cache_ab.py server steps at TP shard sizes 1 2 4 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 python -u - > gpurun_out/dgrad_check.txt 2>&1 <<'PY' || { echo CHECK_FAIL; tail -20 gpurun_out/dgrad_check.txt; exit 1; }
import torch
from splitlearning_amd import ops
from splitlearning_amd.ops import hip_ops as H
ops.set_backend("hip")
C = H.C(); dev = torch.device("cuda", 0); torch.manual_seed(0)
for K in (5000, 2500, 1252, 628):
    dz = torch.randn(16, 1000, device=dev); w = torch.randn(1000, K, device=dev) * 0.02
    h = torch.randn(16, K, device=dev)
    ref = torch.where(h > 0, (dz.double() @ w.double()) * 2.0, torch.zeros((), dtype=torch.float64, device=dev))
    for v in (0, 1, 16, 32, 64):
        C.set_variant(5, v)
        out = H.linear_dgrad(dz, w, h, 2.0)
        err = (out.double() - ref).abs().max().item()
        print(f"K={K} variant5={v} maxerr={err:.3e}", flush=True)
        assert err < 1e-3, err
C.set_variant(5, 0)
print("dgrad check ok")
PY
tail -1 gpurun_out/dgrad_check.txt
timeout -k 10 500 python -u scripts/cache_ab.py --tp 1 2 4 8 --variants ${AB_VARIANTS:-zz+wt dgS16 dgS32 dgS64} ${AB_ARGS} > gpurun_out/dgrad_ab.txt 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/dgrad_ab.txt; exit 1; }
cat gpurun_out/dgrad_ab.txt
