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


def ipc_allreduce(ipc):
    """The TailEngine all-reduce hook over a bare `_C.IpcAllReduce` (no RCCL communicator:
    ranks that share one GPU).  Not capturable (the flag generation is a launch argument)."""
    def _ar(t: torch.Tensor):
        ipc.allreduce_sum(t)
        return t
    _ar.capturable = False
    _ar.ipc = ipc             # the native executor (engine.ServerEpoch) issues it from C++
    return _ar


def native_allreduce(tpc):
    def _ar(t: torch.Tensor):
        tpc.allreduce_sum(t)
        return t
    _ar.capturable = True
    _ar.comm = tpc            # the native executor (engine.ServerEpoch) issues it from C++
    return _ar


# Largest all-reduce the peer-mapped path serves (floats): Bob's row-parallel fc2 partial is
# B x 1000 (64 x 1000 at the largest fused batch); anything larger goes to RCCL.
IPC_AR_CAP = 64 * 1024


def _agree(flag: bool, group=None) -> bool:
    """Every process learns whether `flag` holds on all of them (MIN all-reduce)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def ipc_self_test(ipc, iters: int = 24) -> bool:
    """Run the peer-mapped all-reduce on known data (every size class it serves, both parity
    buffers many times over) and check every element against the fixed-order sum.  The
    values are small multiples of 1/2, so the fp32 sums are exact."""
    T, me = ipc.size, ipc.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    old = 30.0
    ipc.set_timeout_s(5.0)                 # a broken mapping fails the test, not the job
    try:
        for it in range(iters):
            n = (16 * 1000, 4, 1028, ipc.cap)[it % 4]
            base = (torch.arange(n, dtype=torch.float32) % 97) * 0.5 + it
            x = (base + (me + 1)).to(dev)
            ipc.allreduce_sum(x)
            want = base * T + T * (T + 1) / 2
            torch.cuda.synchronize(dev)
            if ipc.error() != 0 or not torch.equal(x.cpu(), want):
                return False
        return True
    finally:
        ipc.set_timeout_s(old)


# Outcome of the last peer-mapped set-up on this process (bench.py reports it): "setup" is
# "ok" or the failure, "self_test" True / False / None (not reached), "fallback" the
# all-reduce the job keeps when the peer-mapped path is refused.
IPC_STATUS: dict = {}


def make_ipc_allreduce(ranks: list[int], my_rank: int, cap: int = IPC_AR_CAP, group=None):
    """Collective over every process: a peer-mapped all-reduce (`_C.IpcAllReduce`, csrc/ipc_ar.h)
    among `ranks`, returned on members after set-up (IPC handle exchange, peer mapping) AND a
    self-test passed on every member; None everywhere otherwise (the caller keeps RCCL).
    `group` is the torch.distributed group containing `ranks` (default: the world)."""
    from .. import _native
    C = _native.load()
    member = my_rank in ranks and len(ranks) > 1
    ipc, h, err = None, None, None
    if member:
        try:
            ipc = C.IpcAllReduce(len(ranks), ranks.index(my_rank), cap)
            h = ipc.handle()
        except RuntimeError as e:
            ipc, err = None, e
    world = dist.get_world_size(group)
    hs = [None] * world
    dist.all_gather_object(hs, h, group=group)
    if member and ipc is not None:
        # hs is indexed by group rank; `ranks` are global ranks
        order = dist.get_process_group_ranks(group) if group is not None else list(range(world))
        mine = [hs[order.index(r)] for r in ranks]
        if any(x is None for x in mine):
            err = "a peer could not export its region"
        else:
            try:
                ipc.open(mine)
            except RuntimeError as e:
                err = e
    IPC_STATUS.clear()
    IPC_STATUS.update({"ranks": len(ranks), "setup": "ok" if err is None else str(err)[:200], "self_test": None,
                       "fallback": None})
    if not _agree(err is None, group):
        import warnings
        warnings.warn(f"peer-mapped all-reduce unavailable ({err or 'failed on another rank'}); using RCCL")
        IPC_STATUS.update({"setup": IPC_STATUS["setup"] if err is not None else "failed on another rank",
                           "fallback": "rccl"})
        return None
    ok = True
    if member:
        try:
            ok = ipc_self_test(ipc)
        except RuntimeError:
            ok = False
    agreed = _agree(ok, group)
    IPC_STATUS.update({"self_test": bool(ok and agreed)})
    if not agreed:
        import warnings
        warnings.warn("peer-mapped all-reduce failed its self-test on some rank; using RCCL")
        IPC_STATUS["fallback"] = "rccl"
        return None
    return ipc if member else None


def _channel_self_test(ch, iters: int = 12) -> bool:
    """Ring messages over the channel (rank r -> r + 1), every size class it serves and both
    parity slots several times over, checked element-wise (exact: the values are copied)."""
    T, me = ch.size, ch.rank
    if T < 2:
        return True
    dev = torch.device("cuda", torch.cuda.current_device())
    old = ch.timeout_s
    ch.set_timeout_s(5.0)
    try:
        for it in range(iters):
            n = min((4, 1028, 16 * 5408 + 32, ch.cap)[it % 4], ch.cap)
            src = (me - 1) % T
            out = (torch.arange(n, dtype=torch.float32) * 0.25 + 1000 * me + it).to(dev)
            got = torch.empty(n, device=dev)
            ch.send(out, (me + 1) % T)
            ch.recv(got, src)
            want = torch.arange(n, dtype=torch.float32) * 0.25 + 1000 * src + it
            torch.cuda.synchronize(dev)
            if ch.error() != 0 or not torch.equal(got.cpu(), want):
                return False
        return True
    finally:
        ch.set_timeout_s(old)


# Outcome of the last split-channel set-up on this process (bench.py reports it)
CHANNEL_STATUS: dict = {}


def make_ipc_channel(cap: int, group=None):
    """Collective over every process: a peer-mapped point-to-point channel (`_C.IpcChannel`,
    csrc/ipc_p2p.h) over all ranks, carrying messages of up to `cap` floats — returned after
    set-up AND a ring self-test passed on every rank; None everywhere otherwise."""
    from .. import _native
    C = _native.load()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    ch, h, err = None, None, None
    try:
        ch = C.IpcChannel(world, rank, cap)
        h = ch.handle()
    except RuntimeError as e:
        ch, err = None, e
    hs = [None] * world
    dist.all_gather_object(hs, h, group=group)
    if ch is not None:
        if any(x is None for x in hs):
            err = "a peer could not export its region"
        else:
            try:
                ch.open(hs)
            except RuntimeError as e:
                err = e
    CHANNEL_STATUS.clear()
    CHANNEL_STATUS.update({"kind": "ipc", "setup": "ok" if err is None else str(err)[:200], "self_test": None})
    if not _agree(err is None, group):
        CHANNEL_STATUS["setup"] = CHANNEL_STATUS["setup"] if err is not None else "failed on another rank"
        return None
    try:
        ok = _channel_self_test(ch)
    except RuntimeError:
        ok = False
    agreed = _agree(ok, group)
    CHANNEL_STATUS["self_test"] = bool(ok and agreed)
    return ch if agreed else None
