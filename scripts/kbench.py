"""Kernel microbenchmarks at the flagship shapes (MI355X).  Prints one line per
(kernel, variant) with device time per call and effective HBM GB/s, interleaving
variants in rounds inside one process (guide §5.4 rule 24), plus whole-step timings
of the Bob server step and the Alice local step.

    python scripts/kbench.py [--iters 200] [--rounds 5] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd import ops  # noqa: E402
from splitlearning_amd.config import OptimCfg  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", type=str, default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C = H.C()
    ops.set_backend("hip")
    torch.manual_seed(0)
    M, K1, N1, N2, N3 = 16, 5408, 5000, 1000, 100
    x = torch.rand(M, K1, device=dev) * 10
    W1 = torch.randn(N1, K1, device=dev) * 0.01
    b1 = torch.randn(N1, device=dev)
    W2 = torch.randn(N2, N1, device=dev) * 0.01
    h1 = torch.relu(torch.randn(M, N1, device=dev))
    dz1 = torch.randn(M, N1, device=dev)
    dz2 = torch.randn(M, N2, device=dev)
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5)
    sW1 = {"m": torch.zeros_like(W1), "v": torch.zeros_like(W1)}
    sb1 = {"m": torch.zeros_like(b1), "v": torch.zeros_like(b1)}
    out = torch.empty(M, N1, device=dev)
    res = {}

    def rec(name, us, nbytes):
        res.setdefault(name, []).append(us)

    cases = []
    cases.append(("fc1_fwd", lambda: H.linear_fwd(x, W1, b1, True, 0.5, 7, 0, out=out), W1.numel() * 4))
    cases.append(("fc1_wgrad_adam", lambda: H.linear_wgrad_step_(dz1, x, W1, b1, cfg, sW1, sb1, 3),
                  W1.numel() * 24))
    sW2 = {"m": torch.zeros_like(W2), "v": torch.zeros_like(W2)}
    b2 = torch.zeros(N2, device=dev)
    sb2 = {"m": torch.zeros_like(b2), "v": torch.zeros_like(b2)}
    cases.append(("fc2_wgrad_adam", lambda: H.linear_wgrad_step_(dz2, h1, W2, b2, cfg, sW2, sb2, 3),
                  W2.numel() * 24))
    cases.append(("fc1_dgrad", lambda: H.linear_dgrad(dz1, W1, None, 1.0), W1.numel() * 4))
    cases.append(("fc2_dgrad", lambda: H.linear_dgrad(dz2, W2, h1, 2.0), W2.numel() * 4))
    cases.append(("fc2_fwd", lambda: H.linear_fwd(h1, W2, None, True, 0.5, 7, 0), W2.numel() * 4))
    logits = torch.randn(M, 100, device=dev)
    yl = torch.randint(0, 10, (M,), device=dev)
    cases.append(("ce_100", lambda: H.softmax_ce(logits, yl, 1 / 16), 0))
    act = torch.rand(M, 5408, device=dev)
    cases.append(("ce_5408", lambda: H.softmax_ce(act, yl, 1 / 16), 0))
    shard = torch.randint(0, 256, (4096, 784), device=dev, dtype=torch.uint8)
    ylab = torch.randint(0, 10, (4096,), device=dev)
    idx = torch.randperm(4096, device=dev)[:M]
    cw = torch.randn(32, 1, 3, 3, device=dev) * 0.1
    cb = torch.randn(32, device=dev) * 0.1
    scw = {"m": torch.zeros_like(cw), "v": torch.zeros_like(cw)}
    scb = {"m": torch.zeros_like(cb), "v": torch.zeros_like(cb)}
    cases.append(("conv_fwd", lambda: H.conv_front_fwd(shard, idx, cw, cb), 0))
    cases.append(("conv_local_step(2 kernels)", lambda: H.conv_local_step_(shard, ylab, idx, cw, cb, cfg, scw,
                                                                            scb, 2), 0))
    n_ep = min(2048, shard.shape[0] // 16 * 16)
    order = torch.randperm(shard.shape[0], device=dev)[:n_ep]

    cases.append((f"conv_local_epoch[{n_ep // 16} steps, fused opt]",
                  lambda: H.conv_local_epoch_(shard, ylab, order, 16, cw, cb, cfg, scw, scb, 2), 0))
    y, am = H.conv_front_fwd(shard, idx, cw, cb)
    dy = torch.randn(M, 5408, device=dev)
    cases.append(("conv_bwd_step(2 kernels)", lambda: H.conv_front_bwd_step_(dy, y, am, shard, idx, cw, cb, cfg,
                                                                              scw, scb, 2), 0))
    # whole Bob SISA server step through the engine
    from splitlearning_amd.engine import OptSlot, TailEngine, adam
    from splitlearning_amd.models import ServerTailSisa, sisa_server_spec
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev)
    slot = OptSlot(adam(1e-3, 1e-5))

    def bob_step():
        o = tail.forward(x, train=True)
        _, d = H.softmax_ce(o, yl, 1 / 16)
        tail.backward_dgrad(d, need_dx=False)
        tail.backward_step(slot)
    cases.append(("bob_server_step", bob_step, 32_146_100 * 28))

    def bob_step_dx():
        o = tail.forward(x, train=True)
        _, d = H.softmax_ce(o, yl, 1 / 16)
        tail.backward_dgrad(d, need_dx=True)
        tail.backward_step(slot)
    cases.append(("bob_step_with_dx", bob_step_dx, 32_146_100 * 32))
    ftail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev)
    fslot = OptSlot(adam(1e-3, 1e-5))
    # pieces of the fused step
    L1, L2, L3 = ftail.layers
    h1f = torch.relu(torch.randn(M, N1, device=dev))
    P2 = H.linear_fwd_partial(h1f, L2.W)
    cases.append(("fused:fc2_fwd_partial", lambda: H.linear_fwd_partial(h1f, L2.W), W2.numel() * 4))
    cases.append(("fused:head3", lambda: H.server_head3(P2, L2.b, True, 0.5, 3, L3.W, L3.b, yl, 1 / 16), 0))
    h2f, dlf, dz2f, _ = H.server_head3(P2, L2.b, True, 0.5, 3, L3.W, L3.b, yl, 1 / 16)
    dz1f = H.linear_dgrad(dz2f, L2.W, h1f, 2.0)
    wst = [fslot.state(f"fc{i}.{n}", t) for i, L in ((1, L1), (2, L2), (3, L3)) for n, t in
           (("weight", L.W), ("bias", L.b))]
    grp = [(dz1f, x, L1.W, wst[0], L1.b, wst[1]), (dz2f, h1f, L2.W, wst[2], L2.b, wst[3]),
           (dlf, h2f, L3.W, wst[4], L3.b, wst[5])]
    cases.append(("fused:wgrad_group3", lambda: H.wgrad_group_(grp, M, cfg, 3), 32_146_100 * 24))
    cases.append(("fused:wgrad_fc1_only", lambda: H.wgrad_group_(grp[:1], M, cfg, 3), W1.numel() * 24))
    dz1r = torch.randn(M, N1, device=dev)
    pn = H.lookahead_slabs(dev, 5408, M, N1)
    cases.append(("fused:wgrad_group3_lookahead",
                  lambda: H.wgrad_group_(grp, M, cfg, 3, x_next=x, p_next=pn), 32_146_100 * 24))
    cases.append(("v3:wgrad_fc1_same_tensors", lambda: H.linear_wgrad_step_(dz1r, x, L1.W, L1.b, cfg, wst[0], wst[1], 3),
                  W1.numel() * 24))

    def bob_fused():
        ftail.train_fwd_bwd3(x, yl, need_dx=False)
        ftail.fused_step(fslot)
    cases.append(("bob_fused_step", bob_fused, 32_146_100 * 28))
    ltail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev)
    lslot = OptSlot(adam(1e-3, 1e-5))
    ltail.lookahead_prologue(x)

    def bob_lookahead():
        ltail.train_fwd_bwd3(x, yl, need_dx=False, pre=True)
        ltail.fused_step(lslot, x_next=x)
    cases.append(("bob_lookahead_step", bob_lookahead, 32_146_100 * 24))
    # graph-replayed server steps (per-step time = one replay of 16 steps / 16)
    from splitlearning_amd.engine.graphs import GraphedServerSteps
    gtail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev)
    gslot = OptSlot(adam(1e-3, 1e-5))
    gs = GraphedServerSteps(gtail, gslot, 16, 16, 5408)
    cache_x = torch.rand(16 * 16, 5408, device=dev) * 10
    cache_y = torch.randint(0, 10, (16 * 16,), device=dev)

    class _PerStep:
        def __call__(self):
            gs.run(cache_x, cache_y, 16)
    cases.append(("bob_graph_16steps", _PerStep(), 32_146_100 * 28 * 16))
    bytes_of = {n: b for n, _, b in cases}
    for _ in range(a.rounds):
        for name, fn, nb in cases:
            rec(name, timeit(fn, a.iters), nb)
    table = []
    for name, ts in res.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        gbs = bytes_of[name] / (med * 1e-6) / 1e9 if bytes_of[name] else None
        table.append({"kernel": name, "median_us": round(med, 2), "min_us": round(ts[0], 2),
                      "GBps": round(gbs, 1) if gbs else None})
        print(f"{name:32s} median {med:9.2f} us   min {ts[0]:9.2f} us   " +
              (f"{gbs:8.1f} GB/s" if gbs else ""), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "rows": table}, f, indent=1)


if __name__ == "__main__":
    main()
