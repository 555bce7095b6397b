"""`engine.resident.Failsafe` decisions on CPU (the launch itself is stubbed): a launch that
returns non-finite results is rolled back like one that timed out, and a fatal error on one
Bob rank ends every rank together instead of leaving the others blocked in the agreement.

Reference failure rule: split_nn.py:183-186 (mp.spawn join=True: one child's exception ends
the job)."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from splitlearning_amd.engine import OptSlot, TailEngine, adam
from splitlearning_amd.engine.resident import Failsafe
from splitlearning_amd.models.zoo import LinearSpec, TailSpec, _MLP


def _small(tp_rank=0, tp_size=1):
    spec = TailSpec([LinearSpec("fc1", 32, 24, True, 0.0), LinearSpec("fc2", 24, 16, True, 0.0),
                     LinearSpec("fc3", 16, 10, False, 0.0)])
    torch.manual_seed(0)
    t = TailEngine(_MLP(spec), spec, torch.device("cpu"), tp_rank=tp_rank, tp_size=tp_size)
    s = OptSlot(adam(1e-3, 1e-5))
    for L in t.layers:
        s.state(f"{L.spec.name}.weight", L.W)
        s.state(f"{L.spec.name}.bias", L.b)
    return t, s


class _Ex:
    def set_fault_step(self, k):
        pass


def _stub(t, behaviour):
    """Replace the persistent launch with `behaviour(t, slot)` -> losses."""
    t._hybrid_executor = lambda slot, B: _Ex()

    def run(acts, labels, slot, B, step_rows=None):
        t.fwd_count += acts.shape[0] // B
        slot.t += acts.shape[0] // B
        return behaviour(t, slot, acts)
    t.run_hybrid_epoch = run


def _state(t, s):
    out = [L.W.clone() for L in t.layers] + [L.b.clone() for L in t.layers]
    out += [v.clone() for st in s.states.values() for v in st.values()]
    return out


@pytest.mark.parametrize("where", ["loss", "weight", "state"])
def test_nonfinite_result_rolls_back(where):
    t, s = _small()
    before = _state(t, s)
    counters = (t.fwd_count, s.t)

    def bad(t, slot, acts):
        loss = torch.ones(acts.shape[0])
        t.layers[1].W.add_(0.5)                     # a partial update the rollback must undo
        if where == "loss":
            loss[3] = float("nan")
        elif where == "weight":
            t.layers[0].W[2, 1] = float("inf")
        else:
            slot.state("fc2.bias", t.layers[1].b)["v"][0] = float("nan")
        return loss
    _stub(t, bad)
    fs = Failsafe(t, s, 4)
    assert not fs.run("hybrid", torch.zeros(16, 32), torch.zeros(16, dtype=torch.long))
    assert fs.fallback["epoch"] == 0 and "non-finite" in fs.fallback["reason"]
    after = _state(t, s)
    assert all(torch.equal(a, b) for a, b in zip(before, after))
    assert (t.fwd_count, s.t) == counters


def test_finite_result_is_kept():
    t, s = _small()

    def good(t, slot, acts):
        t.layers[1].W.add_(0.5)
        return torch.ones(acts.shape[0])
    _stub(t, good)
    w = t.layers[1].W.clone()
    fs = Failsafe(t, s, 4)
    assert fs.run("hybrid", torch.zeros(16, 32), torch.zeros(16, dtype=torch.long))
    assert fs.fallback is None and torch.equal(t.layers[1].W, w + 0.5)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _fatal_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=60))
    t, s = _small(rank, world)

    def run(t, slot, acts):
        if rank == 0:
            raise RuntimeError("hybrid epoch launch: invalid configuration")   # not a wait timeout
        return torch.ones(acts.shape[0])
    _stub(t, run)
    fs = Failsafe(t, s, 4, group=None)
    try:
        fs.run("hybrid", torch.zeros(16, 32), torch.zeros(16, dtype=torch.long))
        q.put((rank, "returned"))
    except RuntimeError as e:
        q.put((rank, "raised: " + str(e)[:80]))
    dist.destroy_process_group()


def test_fatal_error_on_one_rank_ends_every_rank():
    """Rank 0's launch raises a non-recoverable error; rank 1's launch finished.  Both join the
    agreement, both raise (rank 1 names the other rank), nobody waits out a collective timeout."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fatal_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(90)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res[0].startswith("raised: hybrid epoch launch"), res
    assert res[1].startswith("raised") and "another Bob rank" in res[1], res
