"""Native RCCL communicators (`_C.TpComm`) bootstrapped over torch.distributed.

The control plane (rendezvous, timeouts, object broadcast) stays with the
torch.distributed process group; the hot data plane — Bob's per-step tensor-parallel
all-reduce — goes through a communicator the C++ side owns, issued on the current
HIP stream, so it can be captured in the server-step HIP graph.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def make_native_comm(ranks: list[int], my_rank: int, group=None):
    """Collective over every process: returns a `_C.TpComm` on members of `ranks`,
    None elsewhere — and None everywhere when any member could not create it (the
    callers then keep the torch.distributed path).  `group` is the torch.distributed group
    containing `ranks`."""
    from .. import _native
    C = _native.load()
    err = None
    uid = None
    if my_rank == ranks[0]:
        try:
            uid = C.nccl_unique_id()
        except RuntimeError as e:
            err = e
    box = [uid]
    dist.broadcast_object_list(box, src=ranks[0], group=group)
    comm = None
    if box[0] is None and err is None:
        err = "no RCCL unique id from rank %d" % ranks[0]
    if my_rank in ranks and box[0] is not None:
        try:
            comm = C.TpComm(box[0], len(ranks), ranks.index(my_rank))
        except RuntimeError as e:           # e.g. an RCCL the process cannot initialise
            err = e
    # every rank agrees: if any member failed, nobody uses a native communicator and the
    # caller keeps the torch.distributed path (same protocol, Python-issued)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if int(ok.item()) == 0:
        import warnings
        warnings.warn(f"native RCCL communicator unavailable ({err or 'failed on another rank'}); "
                      "using torch.distributed p2p / collectives")
        return None
    return comm


def self_comm():
    """A 1-rank communicator (tests / single-GPU graph capture of the collective path)."""
    from .. import _native
    C = _native.load()
    return C.TpComm(C.nccl_unique_id(), 1, 0)


def native_allreduce(tpc):
    def _ar(t: torch.Tensor):
        tpc.allreduce_sum(t)
        return t
    _ar.capturable = True
    _ar.comm = tpc            # the native executor (engine.ServerEpoch) issues it from C++
    return _ar
