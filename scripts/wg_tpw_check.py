"""wgrad_group with two tiles per workgroup (variant 22 = 1) against one (the shipped form):
the parameters, optimizer state and look-ahead slabs must be bitwise equal (same per-tile
arithmetic, only the issue order differs).  Prints OK / the first mismatch per case."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.config import OptimCfg  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def run(case, var):
    C = H.C()
    C.set_variant(22, var)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    M = 16
    if case == "ushape":
        shapes, cfg = [(1000, 5408), (100, 1000)], OptimCfg("adam", 1e-3, weight_decay=1e-5)
    elif case == "vanilla":
        shapes, cfg = [(5000, 5408), (1000, 5000), (100, 1000)], OptimCfg("sgd", 1e-2, momentum=0.9)
    else:   # a TP = 8 SISA shard: fc1 628 x 5408 (Adam)
        shapes, cfg = [(628, 5408), (1000, 628), (100, 1000)], OptimCfg("adam", 1e-3, weight_decay=1e-5)
    adam = cfg.kind == "adam"
    Ls = []
    for n, k in shapes:
        W = (torch.randn(n, k, generator=g) * 0.01).to(dev)
        b = torch.randn(n, generator=g).to(dev)
        st = ({"m": torch.randn(n, k, generator=g).to(dev) * 1e-3, "v": torch.rand(n, k, generator=g).to(dev) * 1e-6}
              if adam else {"buf": torch.randn(n, k, generator=g).to(dev) * 1e-3})
        sb = {kk: torch.zeros(n, device=dev) for kk in st}
        Ls.append((torch.randn(M, n, generator=g).to(dev), torch.rand(M, k, generator=g).to(dev), W, st, b, sb))
    xn = torch.rand(M, shapes[0][1], generator=g).to(dev)
    pn = H.lookahead_slabs(dev, shapes[0][1], M, shapes[0][0]).clone()
    for t in (1, 2):
        H.wgrad_group_(Ls, M, cfg, t, x_next=xn, p_next=pn)
    torch.cuda.synchronize()
    C.set_variant(22, 0)
    out = [pn]
    for (_, _, W, st, b, sb) in Ls:
        out += [W, b] + list(st.values()) + list(sb.values())
    return out


def main():
    for case in ("ushape", "vanilla", "tp8"):
        a, b = run(case, 0), run(case, 1)
        bad = [i for i, (x, y) in enumerate(zip(a, b)) if not torch.equal(x, y)]
        print(f"{case}: {'OK' if not bad else 'MISMATCH in tensors ' + str(bad)}", flush=True)
        if bad:
            sys.exit(1)


if __name__ == "__main__":
    main()
