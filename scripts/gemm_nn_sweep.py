"""Split-K sweep of the NN data-gradient GEMM (csrc/gemm.hip gemm_nn_dgrad, dX = mask(dZ . W)) at
the evaluation / large-batch shapes, against torch.mm (hipBLASLt) on the same product:

    python scripts/gemm_nn_sweep.py [--splits 0 1 2 3 4 5 6 8 10 12 16] [--reps 20]

Split 0 = the kernel's own choice.  Each point is checked against torch (relative error).
Reference op: the backward of nn.Linear over --batch_size rows (data_entities_vanilla.py:231).
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def bench(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", type=int, nargs="+", default=[0, 1, 2, 3, 4, 5, 6, 8, 10, 12, 16])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--M", type=int, nargs="+", default=[200, 1000])
    ap.add_argument("--form", type=int, default=0, help="0: the kernel's choice of tile; 2: 128 x 128; 4: 256 x 128")
    ap.add_argument("--nt", action="store_true", help="the forward (NT) product Y = X W^T instead (gemm_nt)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C = H.C()
    C.set_gemm_nn_form(a.form)
    if a.nt:
        return sweep_nt(a, C, dev)
    for M in a.M:
        for N, K in ((5000, 5408), (1000, 5000)):
            torch.manual_seed(0)
            dz = torch.randn(M, N, device=dev)
            w = torch.randn(N, K, device=dev) / N ** 0.5
            h = torch.relu(torch.randn(M, K, device=dev))
            ref = torch.where(h > 0, (dz @ w) * 2.0, torch.zeros(1, device=dev))
            fl = 2.0 * M * N * K
            t_mm = bench(lambda: torch.mm(dz, w), a.reps)
            ws = torch.empty(16 * M * K, device=dev)
            out = torch.empty(M, K, device=dev)
            line = [f"form {a.form} M={M} N={N} K={K}: torch.mm {fl / t_mm / 1e12:6.1f} TF"]
            for S in a.splits:
                C.set_gemm_nn_splits(S)
                C.gemm_nn_dgrad(dz, w, h, 2.0, out, ws)
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                t = bench(lambda: C.gemm_nn_dgrad(dz, w, h, 2.0, out, ws), a.reps)
                line.append(f"S{S}: {fl / t / 1e12:5.1f} TF ({100 * t_mm / t:3.0f} %{', ERR %.1e' % err if err > 1e-4 else ''})")
            C.set_gemm_nn_splits(0)
            print(" | ".join(line), flush=True)


def sweep_nt(a, C, dev):
    """gemm_nt's small-grid split over K (Y[M, N] = X[M, K] W[N, K]^T, bias + ReLU fused)."""
    for M in a.M:
        for N, K in ((5000, 5408), (1000, 5000)):
            torch.manual_seed(0)
            x = torch.randn(M, K, device=dev)
            w = torch.randn(N, K, device=dev) / K ** 0.5
            b = torch.randn(N, device=dev)
            ref = torch.relu(x @ w.t() + b)
            fl = 2.0 * M * N * K
            t_mm = bench(lambda: torch.mm(x, w.t()), a.reps)
            line = [f"NT M={M} N={N} K={K}: torch.mm {fl / t_mm / 1e12:6.1f} TF"]
            for S in a.splits:
                C.set_gemm_nt_splits(S)
                y = H.linear_fwd(x, w, b, True, 0.0, 1)
                err = ((y - ref).abs().max() / ref.abs().max()).item()
                t = bench(lambda: H.linear_fwd(x, w, b, True, 0.0, 1), a.reps)
                line.append(f"S{S}: {fl / t / 1e12:5.1f} TF ({100 * t_mm / t:3.0f} %{', ERR %.1e' % err if err > 1e-4 else ''})")
            C.set_gemm_nt_splits(0)
            print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
