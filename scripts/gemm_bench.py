"""Large-M GEMM (csrc/gemm.hip, Y = epi(X W^T)) against torch.mm (hipBLASLt) on Bob's
evaluation shapes, every tile variant (slot 10)."""
import os
import sys
import time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.ops import hip_ops as H  # noqa

dev = torch.device("cuda", 0)
C = H.C()


def bench(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


for M, N, K in [(14000, 5000, 5408), (14000, 1000, 5000), (4096, 4096, 4096)]:
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev)
    b = torch.randn(N, device=dev)
    fl = 2.0 * M * N * K
    t_mm = bench(lambda: torch.mm(x, w.t()))
    xb, wb = x.bfloat16(), w.bfloat16()
    t_mmb = bench(lambda: torch.mm(xb, wb.t()))
    line = [f"M={M} N={N} K={K}: torch.mm fp32 {fl/t_mm/1e12:.1f} TF, bf16 {fl/t_mmb/1e12:.1f} TF"]
    C.set_variant(11, 1)                  # the in-tree GEMM for fp32 too
    for dt in ("fp32", "bf16"):
        C.set_compute_dtype(dt)
        t = bench(lambda: H.linear_fwd(x, w, b, True, 0.0, 0))
        line.append(f"ours {dt} {fl/t/1e12:.1f} TF")
    C.set_variant(11, 0)
    C.set_compute_dtype("fp32")
    print(" | ".join(line), flush=True)
