"""wgrad+optimizer microbenchmark at Bob's tensor-parallel shard sizes (MI355X).

For each TP degree T the fc1 shard is [ceil(5000/T), 5408], fc2's [1000, ceil(5000/T)], fc3
replicated.  Prints device us/call (CUDA events over back-to-back calls, so the shard's
state is as cache-warm as in the real step loop) for:
  stream      opt_flat over the fc1 shard (p, g, m, v read; p, m, v written: 28 B/param) —
              a plain streaming roofline for the same parameter count;
  fc1         wgrad_group over fc1 alone (24 B/param);
  fc1+la      the same plus the look-ahead forward of the next batch;
  group+la    fc1 + fc2 + fc3 + look-ahead (what the server step launches).

    python scripts/wgbench.py [--tps 1 2 4 8] [--iters 100] [--variant 3=1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd.config import OptimCfg  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tps", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--case", choices=("tp", "ushape", "vanilla", "concat", "concat_tp8"), default="tp",
                    help="tp: the SISA tail's shards; ushape: fc1 1000 x 5408 + fc2 100 x 1000 (Adam); "
                         "vanilla: 5000 x 5408 / 1000 x 5000 / 100 x 1000 (SGD-momentum); concat: "
                         "fc1 5000 x 43264 (k = 8, Adam); concat_tp8: its TP = 8 shard (fc1 625 x 43264, fc2 "
                         "1000 x 625, fc3 800 x 1000)")
    a = ap.parse_args()
    if a.case != "tp":
        return other_case(a)
    C = H.C()
    for kv in a.variant:
        slot, val = (int(v) for v in kv.split("="))
        C.set_variant(slot, val)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M, K1, N2, N3 = 16, 5408, 1000, 100
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5)

    def layer(n, k):
        W = torch.randn(n, k, device=dev) * 0.01
        b = torch.zeros(n, device=dev)
        return W, {"m": torch.zeros_like(W), "v": torch.zeros_like(W)}, b, {"m": torch.zeros_like(b),
                                                                           "v": torch.zeros_like(b)}

    for T in a.tps:
        n1 = -(-5000 // T)
        n1 = -(-n1 // 4) * 4
        x = torch.rand(M, K1, device=dev)
        xn = torch.rand(M, K1, device=dev)
        h1 = torch.rand(M, n1, device=dev)
        h2 = torch.rand(M, N2, device=dev)
        dz1 = torch.randn(M, n1, device=dev)
        dz2 = torch.randn(M, N2, device=dev)
        dz3 = torch.randn(M, N3, device=dev)
        W1, s1, b1, sb1 = layer(n1, K1)
        W2, s2, b2, sb2 = layer(N2, n1)
        W3, s3, b3, sb3 = layer(N3, N2)
        g1 = torch.randn_like(W1)
        pn = H.lookahead_slabs(dev, K1, M, n1)
        L1 = (dz1, x, W1, s1, b1, sb1)
        L2 = (dz2, h1, W2, s2, b2, sb2)
        L3 = (dz3, h2, W3, s3, b3, sb3)
        st = {"m": s1["m"], "v": s1["v"]}
        n_par = W1.numel()
        res = {
            "stream": timeit(lambda: H.apply_update_(W1.view(-1), g1.view(-1), {"m": st["m"].view(-1),
                                                                               "v": st["v"].view(-1)}, cfg, 5),
                             a.iters),
            "fc1": timeit(lambda: H.wgrad_group_([L1], M, cfg, 5), a.iters),
            "fc1+la": timeit(lambda: H.wgrad_group_([L1], M, cfg, 5, x_next=xn, p_next=pn), a.iters),
            "group+la": timeit(lambda: H.wgrad_group_([L1, L2, L3], M, cfg, 5, x_next=xn, p_next=pn), a.iters),
        }
        gb = {"stream": 28 * n_par, "fc1": 24 * n_par, "fc1+la": 24 * n_par,
              "group+la": 24 * (n_par + W2.numel() + W3.numel())}
        for k, us in res.items():
            print(f"tp={T} {k:9s} {us:8.2f} us  {gb[k] / us / 1e3:7.0f} GB/s", flush=True)


def other_case(a):
    """wgrad_group over the split modes' / concat's layers, with the look-ahead: us per call and
    the state bytes moved (W + states read and written) per us."""
    C = H.C()
    for kv in a.variant:
        slot, val = (int(v) for v in kv.split("="))
        C.set_variant(slot, val)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = 16
    if a.case == "ushape":
        shapes, cfg = [(1000, 5408), (100, 1000)], OptimCfg("adam", 1e-3, weight_decay=1e-5)
    elif a.case == "vanilla":
        shapes, cfg = [(5000, 5408), (1000, 5000), (100, 1000)], OptimCfg("sgd", 1e-2, momentum=0.9)
    elif a.case == "concat_tp8":
        shapes, cfg = [(628, 43264), (1000, 628), (800, 1000)], OptimCfg("adam", 1e-3, weight_decay=1e-5)
    else:
        shapes, cfg = [(5000, 43264), (1000, 5000), (800, 1000)], OptimCfg("adam", 1e-3, weight_decay=1e-5)
    adam = cfg.kind == "adam"
    Ls, nbytes = [], 0
    for n, k in shapes:
        W = torch.randn(n, k, device=dev) * 0.01
        b = torch.zeros(n, device=dev)
        st = {"m": torch.zeros_like(W), "v": torch.zeros_like(W)} if adam else {"buf": torch.zeros_like(W)}
        sb = {"m": torch.zeros_like(b), "v": torch.zeros_like(b)} if adam else {"buf": torch.zeros_like(b)}
        Ls.append((torch.randn(M, n, device=dev), torch.rand(M, k, device=dev), W, st, b, sb))
        nbytes += W.numel() * 4 * 2 * (3 if adam else 2)
    xn = torch.rand(M, shapes[0][1], device=dev)
    pn = H.lookahead_slabs(dev, shapes[0][1], M, shapes[0][0])
    us = timeit(lambda: H.wgrad_group_(Ls, M, cfg, 5, x_next=xn, p_next=pn), a.iters)
    print(f"{a.case} variants {a.variant}: {us:8.2f} us  {nbytes / us / 1e3:7.0f} GB/s of state traffic", flush=True)
    n1b = Ls[0][2].numel() * 4 * 2 * (3 if adam else 2)
    u1 = timeit(lambda: H.wgrad_group_(Ls[:1], M, cfg, 5), a.iters)
    u2 = timeit(lambda: H.wgrad_group_(Ls[:1], M, cfg, 5, x_next=xn, p_next=pn), a.iters)
    print(f"  fc1 alone: {u1:8.2f} us  {n1b / u1 / 1e3:7.0f} GB/s;  fc1 + look-ahead: {u2:8.2f} us  "
          f"{n1b / u2 / 1e3:7.0f} GB/s", flush=True)
    if a.case == "concat":
        # ceilings for the same bytes: a device copy of W (read + write) and the plain
        # optimizer stream (opt_flat: p, g, m, v read; p, m, v written) over fc1
        W1, st1 = Ls[0][2], Ls[0][3]
        dst = torch.empty_like(W1)
        cu = timeit(lambda: dst.copy_(W1), a.iters)
        print(f"  copy of fc1 W ({W1.numel() * 4 / 1e6:.0f} MB): {cu:8.2f} us  {2 * W1.numel() * 4 / cu / 1e3:7.0f} GB/s",
              flush=True)
        g1 = torch.randn_like(W1)
        so = timeit(lambda: H.apply_update_(W1.view(-1), g1.view(-1), {"m": st1["m"].view(-1), "v": st1["v"].view(-1)},
                                            cfg, 5), a.iters)
        print(f"  opt_flat over fc1: {so:8.2f} us  {28 * W1.numel() / so / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
