"""Large-M GEMM (csrc/gemm.hip, Y = epi(X W^T)) against torch.mm (hipBLASLt) on Bob's
evaluation shapes (fc1 / fc2 / fc3 of model2_sisa at M = 200 / 1000 / 14000 rows) and 4096^3:
fp32 tile forms (slot 10: 0 = the default routing (32x32x2 MFMA, 256 x 128 tiles, or 128 x 128
tiles split over K for small grids); 1..4 = 32x32x2 with (WM, BK) = (2, 16) (4, 16) (2, 32)
(4, 32), no split; 5 = 16x16x4, 256 x 128), checked against torch, plus the bf16 form.

    python scripts/gemm_bench.py [--forms 0 1 2 3 4] [--reps 8] [--dgrad]

`--dgrad`: the data-gradient product dX = dZ . W (NN layout, csrc/gemm.hip gemm_nn_dgrad, the
previous layer's ReLU mask fused) against torch.mm(dZ, W) on the same shapes.
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
    ap.add_argument("--forms", type=int, nargs="+", default=[0, 2, 5])
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--shapes", default="all", choices=("all", "eval", "big"))
    ap.add_argument("--dgrad", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C = H.C()
    shapes = []
    if a.shapes in ("all", "eval"):
        for M in (200, 1000, 14000):
            shapes += [(M, 5000, 5408), (M, 1000, 5000), (M, 100, 1000)]
    if a.shapes in ("all", "big"):
        shapes.append((4096, 4096, 4096))
    if a.dgrad:
        for M, N, K in shapes:
            # forward Y[M, N] = X[M, K] W[N, K]^T  ->  its data gradient dX[M, K] = dY[M, N] W[N, K]
            torch.manual_seed(0)
            dz = torch.randn(M, N, device=dev)
            w = torch.randn(N, K, device=dev) / N ** 0.5
            h = torch.relu(torch.randn(M, K, device=dev))
            fl = 2.0 * M * N * K
            ref = torch.where(h > 0, (dz @ w) * 2.0, torch.zeros(1, device=dev))
            t_mm = bench(lambda: torch.mm(dz, w), a.reps)
            y = H.linear_dgrad(dz, w, h, 2.0)
            err = ((y - ref).abs().max() / ref.abs().max()).item()
            t = bench(lambda: H.linear_dgrad(dz, w, h, 2.0), a.reps)
            print(f"dgrad M={M} N={N} K={K}: torch.mm fp32 {fl / t_mm / 1e12:.1f} TF | in-tree NN (mask fused) "
                  f"{fl / t / 1e12:.1f} TF ({100 * t_mm / t:.0f} %, rel err {err:.1e})", flush=True)
        return
    for M, N, K in shapes:
        torch.manual_seed(0)
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        fl = 2.0 * M * N * K
        ref = torch.relu(x @ w.t() + b)
        t_mm = bench(lambda: torch.mm(x, w.t()), a.reps)
        line = [f"M={M} N={N} K={K}: torch.mm fp32 {fl / t_mm / 1e12:.1f} TF"]
        C.set_variant(11, 1)                  # the in-tree GEMM for fp32 too
        try:
            for f in a.forms:
                C.set_variant(10, f)
                y = H.linear_fwd(x, w, b, True, 0.0, 0)
                err = (y - ref).abs().max().item()
                t = bench(lambda: H.linear_fwd(x, w, b, True, 0.0, 0), a.reps)
                line.append(f"form {f} {fl / t / 1e12:.1f} TF ({100 * t_mm / t:.0f} %, err {err:.1e})")
            C.set_variant(10, 0)
            C.set_compute_dtype("bf16")
            t = bench(lambda: H.linear_fwd(x, w, b, True, 0.0, 0), a.reps)
            line.append(f"bf16 {fl / t / 1e12:.1f} TF")
        finally:
            C.set_variant(10, 0)
            C.set_variant(11, 0)
            C.set_compute_dtype("fp32")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
