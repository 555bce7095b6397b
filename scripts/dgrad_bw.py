"""The vanilla cut-gradient product dx = dz1 . W1 (M = 16, N = 5000, K = 5408: one 108 MB read
of fc1) on the in-tree skinny dgrad against torch.mm (hipBLASLt) and plain reads of W1.

    python scripts/dgrad_bw.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def timeit(fn, iters=200):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M, N, K = 16, 5000, 5408
    W = torch.randn(N, K, device=dev)
    dz = torch.randn(M, N, device=dev)
    gb = N * K * 4 / 1e9
    out = torch.empty_like(W)
    for r in range(3):
        t_ours = timeit(lambda: H.linear_dgrad(dz, W, None, 1.0))
        t_mm = timeit(lambda: torch.mm(dz, W))
        t_sum = timeit(lambda: W.sum(dim=0))
        t_cp = timeit(lambda: out.copy_(W))
        print(f"round {r}: in-tree dgrad {t_ours:.1f} us ({gb / t_ours * 1e3:.2f} TB/s) | torch.mm {t_mm:.1f} us "
              f"({gb / t_mm * 1e3:.2f}) | W.sum(0) {t_sum:.1f} us ({gb / t_sum * 1e3:.2f}) | copy {t_cp:.1f} us "
              f"({2 * gb / t_cp * 1e3:.2f} TB/s r+w)", flush=True)


if __name__ == "__main__":
    main()
