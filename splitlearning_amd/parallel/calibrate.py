"""Link calibration: measured per-message cost of the split-mode data plane and of Bob's TP
all-reduce, on the job's own ranks and transport.

The reference pays ~4 RPC round trips per vanilla batch (activation + labels
out, dist-autograd gradient back, remote optimizer step, context cleanup;
/root/reference/data_entities_vanilla.py:70-76).  Here a batch costs one packed activation
message Alice -> Bob and one cut-gradient message back; on an 8 x MI355X node those cross one
xGMI link each, and their latency (not bandwidth: 346 KB is ~2 us of wire) is what the
Bob tensor-parallel policy trades against the optimizer stream it shards
(`dist.choose_bob_tp`).  `measure` times exactly those messages through the production
`Comm` primitives (the native RCCL communicator on GPUs, torch.distributed / gloo on CPU) as
ping-pongs between rank 0 (Bob's root) and every other rank, plus the TP all-reduce of one
step's fc2 partial (B x 1000 floats) through the tail's all-reduce hook (the peer-mapped
kernel when it passed set-up, else RCCL).  Collective over all ranks; every rank gets rank
0's result.
"""
from __future__ import annotations

import statistics
import time

import torch

from ..config import CUT_FEATURES


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def measure(comm, device, B: int = 16, iters: int = 20, warmup: int = 3, allreduce=None, tp_ranks=()) -> dict:
    """One-way message time per peer (half an act-out / grad-back round trip, us), its median
    (`msg_us`), and the TP all-reduce time per call (`tp_allreduce_us`, when `allreduce` and
    the Bob ranks `tp_ranks` are given; every Bob rank must pass the same hook)."""
    if not comm.distributed:
        return {}
    n_pkt, n_grad = B * CUT_FEATURES + 2 * B, B * CUT_FEATURES   # labels as int64 words (Session.pack)
    pkt = torch.ones(n_pkt, device=device)
    grad = torch.ones(n_grad, device=device)
    per_peer = {}
    for r in range(1, comm.world):
        if comm.rank in (0, r):
            def round_trip():
                comm.send_recv(pkt if comm.rank == r else None, r, 0, (n_pkt,), torch.float32)   # act + labels
                comm.send_recv(grad if comm.rank == 0 else None, 0, r, (n_grad,), torch.float32)  # cut gradient
            for _ in range(warmup):
                round_trip()
            _sync(device)
            t0 = time.perf_counter()
            for _ in range(iters):
                round_trip()
            _sync(device)
            per_peer[r] = (time.perf_counter() - t0) / iters / 2 * 1e6
        comm.barrier()
    ar_us = None
    if allreduce is not None and len(tp_ranks) > 1:
        x = torch.zeros(B * 1000, device=device)
        if comm.rank in tp_ranks:
            for _ in range(warmup):
                allreduce(x)
            _sync(device)
        comm.barrier()
        if comm.rank in tp_ranks:
            t0 = time.perf_counter()
            for _ in range(iters):
                allreduce(x)
            _sync(device)
            ar_us = (time.perf_counter() - t0) / iters * 1e6
        comm.barrier()
    out = {"msg_us": round(statistics.median(per_peer.values()), 2) if per_peer else None,
           "per_peer_us": {int(k): round(v, 2) for k, v in per_peer.items()},
           "tp_allreduce_us": round(ar_us, 2) if ar_us is not None else None,
           "message_floats": {"act_labels": n_pkt, "cut_grad": n_grad}, "iters": iters}
    return comm.broadcast_obj(out, 0)
