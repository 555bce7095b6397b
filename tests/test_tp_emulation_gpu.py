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


@pytest.mark.parametrize("T", [2, 4, 8])
def test_tp_emulated_native_epoch_matches_single_shard(cuda, T):
    B = 16
    steps = 72                                            # >= 64 Adam steps, plus a partial batch
    n = B * steps + 9
    acts, labels = _data(cuda, n)
    torch.manual_seed(0)
    base = ServerTailSisa()
    lr = 1e-3

    ref = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=777)
    rslot = OptSlot(adam(lr, 1e-5))
    assert ref.native_epoch_ok(B)
    ref.lookahead_prologue(acts[:B])
    loss_ref = ref.run_native_epoch(acts, labels, rslot, B, True)

    shards = [TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, tp_rank=r, tp_size=T, allreduce=None,
                         seed_base=777, ws_tag=f"#emu{T}.{r}") for r in range(T)]
    slots = [OptSlot(adam(lr, 1e-5)) for _ in range(T)]
    assert shards[0].layers[0].style == "col" and shards[0].layers[1].style == "row"
    loss = TailEngine.emulate_tp_epoch(shards, slots, acts, labels, B)
    torch.cuda.synchronize()

    assert (shards[0].fwd_count, slots[0].t) == (ref.fwd_count, rslot.t) == (steps + 1, steps + 1)
    # the first step sees identical weights: losses agree to summation-order rounding
    torch.testing.assert_close(loss[:B], loss_ref[:B], rtol=1e-5, atol=1e-5)
    # the trajectory stays on the single-shard one (row-parallel fc2 only reorders the sum)
    torch.testing.assert_close(loss, loss_ref, rtol=2e-3, atol=2e-3)
    # fc3 is replicated: every shard holds bitwise the same copy (same all-reduced inputs)
    for sh in shards[1:]:
        assert torch.equal(sh.layers[2].W, shards[0].layers[2].W)
    for (Wa, ba), Lr in zip(_full(shards), ref.layers):
        for a, b in ((Wa, Lr.W), (ba, Lr.b)):
            d = (a - b).abs()
            assert a.shape == b.shape
            # Adam normalises the update, so elements with ~0 gradients move by up to lr on
            # rounding noise; everything else must agree closely (assert_adam_close form)
            assert d.max().item() <= 2 * lr * (steps + 1) + 1e-6
            assert (d > 1e-4).float().mean().item() < 1e-3


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
