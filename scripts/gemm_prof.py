"""One GEMM shape on the in-tree kernel, repeated (for rocprofv3 counter passes).

    python scripts/gemm_prof.py M N K [reps] [nt|nn]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    form = sys.argv[5] if len(sys.argv) > 5 else "nt"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if form == "nt":
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        H.C().set_variant(11, 1)
        for _ in range(reps):
            H.linear_fwd(x, w, b, True, 0.0, 0)
    else:
        dz = torch.randn(M, N, device=dev)
        w = torch.randn(N, K, device=dev) / N ** 0.5
        h = torch.relu(torch.randn(M, K, device=dev))
        for _ in range(reps):
            H.linear_dgrad(dz, w, h, 2.0)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
