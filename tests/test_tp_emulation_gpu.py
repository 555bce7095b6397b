"""Tensor-parallel Bob through the PRODUCTION native executor, emulated in one process.

The 8-GPU node runs Bob's server epoch as T shard executors (`_C.ServerEpoch`, one per
GPU) with a native RCCL all-reduce of the row-parallel fc2 products.  One GPU cannot host
two RCCL ranks, so `_C.tp_emulate_epoch` steps T shard executors in lock step on one GPU
and stands in for the all-reduce with a fixed-order sum: every other launch is exactly
the production code.  The trajectory must match the single-shard (TP = 1) executor.

Reference semantics: bob.train_and_backward's loop (data_entities_vanilla_sisa.py:298-313).
"""
import copy

import pytest
import torch

from splitlearning_amd.engine import OptSlot, TailEngine, adam
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec

pytestmark = pytest.mark.gpu


def _data(cuda, n, seed=11):
    g = torch.Generator().manual_seed(seed)
    acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    return acts, labels


def _full(shards):
    """Reference-layout weights from the shards (fc1 column-, fc2 row-parallel, fc3 replicated)."""
    L = [sh.layers for sh in shards]
    W1 = torch.cat([l[0].W for l in L], 0)
    b1 = torch.cat([l[0].b for l in L], 0)
    W2 = torch.cat([l[1].W for l in L], 1)
    return [(W1, b1), (W2, L[0][1].b), (L[0][2].W, L[0][2].b)]


def _sync_shards(ref, rslot, shards, slots):
    """Every shard := its slice of the TP = 1 reference's weights, biases and optimizer moments."""
    from splitlearning_amd.engine.tail import _shard_range
    with torch.no_grad():
        for sh, sl in zip(shards, slots):
            for Lr, L in zip(ref.layers, sh.layers):
                for kind, full, mine in (("weight", Lr.W, L.W), ("bias", Lr.b, L.b)):
                    name = f"{Lr.spec.name}.{kind}"
                    pairs = [(full, mine)] + [(rslot.states[name][k], sl.state(name, mine)[k])
                                              for k in rslot.states[name]]
                    for src, dst in pairs:
                        if L.style == "col":
                            s, e = _shard_range(full.shape[0], sh.tp_rank, sh.tp_size)
                            src = src[s:e]
                        elif L.style == "row" and kind == "weight":
                            s, e = _shard_range(full.shape[1], sh.tp_rank, sh.tp_size)
                            src = src[:, s:e]
                        dst.copy_(src)


@pytest.mark.parametrize("T", [2, 4, 8])
@pytest.mark.parametrize("scale", [1.0, 30.0])
def test_tp_emulated_native_epoch_matches_single_shard(cuda, T, scale):
    """72 Adam steps of the native executor at TP = T (emulated) against TP = 1, as 36 two-step
    epochs (look-ahead prologue, the wgrad kernel's look-ahead for the second batch, its
    consumption) each started from the same state: the shards are re-synchronised to the
    TP = 1 run before every pair.  Free-running fp32 trajectories of this random-label
    training are chaotic (any summation-order change grows to O(1) loss gaps within tens of
    steps), so re-synchronisation is what keeps a tight per-step comparison meaningful."""
    B, pairs, lr = 16, 36, 1e-3
    acts, labels = _data(cuda, 2 * B * pairs)
    acts = acts * (scale / 30.0)
    torch.manual_seed(0)
    base = ServerTailSisa()
    ref = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=777)
    rslot = OptSlot(adam(lr, 1e-5))
    for L in ref.layers:
        rslot.state(f"{L.spec.name}.weight", L.W)
        rslot.state(f"{L.spec.name}.bias", L.b)
    shards = [TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, tp_rank=r, tp_size=T, allreduce=None,
                         seed_base=777, ws_tag=f"#emu{T}.{r}") for r in range(T)]
    slots = [OptSlot(adam(lr, 1e-5)) for _ in range(T)]
    assert shards[0].layers[0].style == "col" and shards[0].layers[1].style == "row"
    for j in range(pairs):
        _sync_shards(ref, rslot, shards, slots)
        a, y = acts[2 * j * B:(2 * j + 2) * B], labels[2 * j * B:(2 * j + 2) * B]
        ref.lookahead_prologue(a[:B])
        loss_ref = ref.run_native_epoch(a, y, rslot, B, True)
        loss = TailEngine.emulate_tp_epoch(shards, slots, a, y, B)
        torch.cuda.synchronize()
        assert (shards[0].fwd_count, slots[0].t) == (ref.fwd_count, rslot.t) == (2 * j + 2, 2 * j + 2)
        torch.testing.assert_close(loss, loss_ref, rtol=1e-4, atol=1e-4)
        # fc3 is replicated: every shard holds bitwise the same copy (same all-reduced inputs)
        for sh in shards[1:]:
            assert torch.equal(sh.layers[2].W, shards[0].layers[2].W)
        for (Wa, ba), Lr in zip(_full(shards), ref.layers):
            for a_, b_ in ((Wa, Lr.W), (ba, Lr.b)):
                d = (a_ - b_).abs()
                # two Adam steps from one state: rounding level, except elements whose
                # gradient is ~0 (sign of m / sqrt(v) is rounding noise: <= 2 lr per step)
                assert d.max().item() <= 4 * lr + 1e-6, (j, d.max().item())
                assert (d > 1e-6).float().mean().item() < 1e-4, (j, (d > 1e-6).float().mean().item())


def test_tp_emulation_shard_equals_tp1_when_T_is_1(cuda):
    """T = 1 through the emulation entry point is bitwise the plain executor."""
    B = 16
    n = B * 10 + 3
    acts, labels = _data(cuda, n, seed=3)
    torch.manual_seed(0)
    base = ServerTailSisa()
    a = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=5)
    sa = OptSlot(adam(1e-3, 1e-5))
    a.lookahead_prologue(acts[:B])
    la = a.run_native_epoch(acts, labels, sa, B, True)
    b = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=5, ws_tag="#emu1")
    sb = OptSlot(adam(1e-3, 1e-5))
    lb = TailEngine.emulate_tp_epoch([b], [sb], acts, labels, B)
    torch.cuda.synchronize()
    assert torch.equal(la, lb)
    for L1, L2 in zip(a.layers, b.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)
