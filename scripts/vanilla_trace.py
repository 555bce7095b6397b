"""Per-phase critical path of the vanilla persistent epoch (csrc/vanilla.hip).

Builds a ws = 2 vanilla session on cuda:0 (synthetic MNIST), times whole epochs of the
persistent executor (us per step, median of --reps epochs), then re-runs one epoch with
every workgroup's phase stamps recorded for 8 steps and prints, per stamp, min / median / max
over the workgroups in us after the step's first stamp.  Stamps (VA_MARK in the kernel):
 0 step top            1 F released (forward partials)   2 F arrived          3 B released (dz2)
 4 dz1 partial out     5 W2 step done                    6 U released (dz1)   7 dz1 + b1 staged
 8 update pass done    9 conv released (cut gradient)   10 conv grads out    11 conv grads summed
12 next batch out     13 next batch released            14 forward pass done 15 forward flushed
"""
import argparse
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["top", "F rel", "F arr", "B rel", "dz1 out", "W2 done", "U rel", "dz1 staged", "upd done",
         "conv rel", "cw out", "cw summed", "x out", "x rel", "fwd done", "fwd flushed"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--trace_step", type=int, default=100)
    a = ap.parse_args()
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    from splitlearning_amd.protocols import split_native as sn
    dev = torch.device("cuda", 0)
    tmp = tempfile.mkdtemp()
    n = a.batches * a.B
    args = parse_args(["--vanilla", "--world_size", "2", "--seed", "3", "--num_samples", str(int(n * 2.6) + 100),
                       "--no_tqdm", "--batch_size", str(a.B), "--datapath", tmp + "/d", "--log_dir", tmp + "/l"])
    write_shards(args, verbose=False)
    s = VanillaSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
    a1 = s.alices[1]
    order = a1.train.shuffled_order(torch.Generator().manual_seed(1))[:n].to(dev)
    assert order.numel() == n, (order.numel(), n)
    assert sn.persistent_vanilla_ok(s, 1), s.__dict__.get("split_persist_reason")
    ts = []
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.split_epoch(1, order, n)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) / a.batches * 1e6)
    ts.sort()
    print(f"vanilla persistent epoch: {a.batches} steps of B = {a.B}: {ts[len(ts) // 2]:.1f} us/step "
          f"(min {ts[0]:.1f}, max {ts[-1]:.1f})", flush=True)
    cfg = sn._va_cfg(s, 1)
    ex = s.ops.C().VanillaEpoch(cfg)
    G, T = 256, 8
    tall = torch.zeros((T, G, 16), dtype=torch.int64, device=dev)
    loss = torch.empty(n, device=dev)
    ex.run(order, loss, 0, 0, 0, 1, tall, a.trace_step)
    torch.cuda.synchronize()
    t = tall.cpu().double() / 100.0   # wall clock 100 MHz -> us
    tab = ex.table().cpu()
    nrb = (s.tail.layers[0].W.shape[0] + 15) // 16
    ncb = (s.tail.layers[0].W.shape[1] + 255) // 256
    oU = G + 1 + 2 * nrb + G // 8
    per = []
    for k in range(T - 1):
        per.append(float(t[k + 1, :, 0].median() - t[k, :, 0].median()))
    print(f"traced step (top to top, median over workgroups): {sorted(per)[len(per) // 2]:.1f} us")
    print(f"{'stamp':>14s} {'min':>8s} {'median':>8s} {'max':>8s}   (us after the step's first 'top')")
    for m in range(16):
        rows = []
        for k in range(T - 1):
            base = t[k, :, 0].min()
            col = t[k, :, m]
            col = col[col > 0]
            if col.numel():
                rows.append(((col.min() - base).item(), (col.median() - base).item(), (col.max() - base).item()))
        if rows:
            mid = sorted(rows, key=lambda x: x[1])[len(rows) // 2]
            print(f"{m:2d} {NAMES[m]:>11s} {mid[0]:8.1f} {mid[1]:8.1f} {mid[2]:8.1f}")
    spread(t[:T - 1], tab, G, nrb, oU)


def spread(t, tab, G, nrb, oU):
    """Stamp 8 (update pass done) relative to stamp 7 per workgroup: by XCD (w % 8) and by run
    shape (tiles, column blocks touched)."""
    import collections
    d = (t[:, :, 8] - t[:, :, 7]).median(dim=0).values   # per workgroup, median over steps
    by_x = collections.defaultdict(list)
    by_shape = collections.defaultdict(list)
    for w in range(G):
        u0, u1 = int(tab[oU + w]), int(tab[oU + w + 1])
        ncbs = (u1 - 1) // nrb - u0 // nrb + 1
        by_x[w % 8].append(float(d[w]))
        by_shape[(u1 - u0, ncbs, u0 // nrb == 21 or (u1 - 1) // nrb == 21)].append(float(d[w]))
    print("update pass (stamp 7 -> 8) by XCD: " + "  ".join(f"{x}: {sorted(v)[len(v) // 2]:.1f}/{max(v):.1f}" for x, v in sorted(by_x.items())))
    for k, v in sorted(by_shape.items()):
        print(f"  run {k[0]} tiles, {k[1]} column block(s), touches the 32-wide block: {k[2]!s:5s} "
              f"n={len(v):3d} median {sorted(v)[len(v) // 2]:.1f} max {max(v):.1f}")
    slow = sorted(range(G), key=lambda w: -float(d[w]))[:8]
    print("slowest: " + ", ".join(f"w{w} ({float(d[w]):.1f})" for w in slow))


if __name__ == "__main__":
    main()
