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
from splitlearning_amd.ops import hip_ops

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


def _gaps(loss, ref, B, steps):
    return torch.stack([(loss[i * B:(i + 1) * B] - ref[i * B:(i + 1) * B]).abs().max() for i in range(steps)])


@pytest.mark.parametrize("T", [2, 4, 8])
@pytest.mark.parametrize("scale", [1.0, 30.0])
def test_tp_emulated_native_epoch_matches_single_shard(cuda, T, scale):
    """72 Adam steps.  Training with random labels is chaotic: ANY change of fp32 summation
    order (e.g. the TP = 1 executor with its other fc2-dgrad form, variant 8 = 2) grows from
    1e-6 to O(1) loss gaps over tens of steps.  So the TP = T run must (a) agree tightly on
    the early steps, where a shard-math bug would already show as O(1) gaps, and (b) stay
    within the rounding-noise envelope of that TP = 1 alternative over the whole run."""
    B = 16
    steps = 72
    n = B * steps
    acts, labels = _data(cuda, n)
    acts = acts * (scale / 30.0)
    torch.manual_seed(0)
    base = ServerTailSisa()
    lr = 1e-3
    C = hip_ops.C()

    def tp1(variant, tag):
        C.set_variant(8, variant)
        try:
            t = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=777, ws_tag=tag)
            s = OptSlot(adam(lr, 1e-5))
            t.lookahead_prologue(acts[:B])
            return t, s, t.run_native_epoch(acts, labels, s, B, True)
        finally:
            C.set_variant(8, 0)
    ref, rslot, loss_ref = tp1(0, "")
    alt, _, loss_alt = tp1(2, "#alt")

    shards = [TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, tp_rank=r, tp_size=T, allreduce=None,
                         seed_base=777, ws_tag=f"#emu{T}.{r}") for r in range(T)]
    slots = [OptSlot(adam(lr, 1e-5)) for _ in range(T)]
    assert shards[0].layers[0].style == "col" and shards[0].layers[1].style == "row"
    loss = TailEngine.emulate_tp_epoch(shards, slots, acts, labels, B)
    torch.cuda.synchronize()

    assert (shards[0].fwd_count, slots[0].t) == (ref.fwd_count, rslot.t) == (steps, steps)
    # (a) early steps: identical weights at step 1, rounding-level gaps for the next ones
    torch.testing.assert_close(loss[:B], loss_ref[:B], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss[:8 * B], loss_ref[:8 * B], rtol=1e-3, atol=1e-3)
    # (b) the whole run inside the TP = 1 rounding-noise envelope
    g_tp, g_alt = _gaps(loss, loss_ref, B, steps), _gaps(loss_alt, loss_ref, B, steps)
    assert g_tp.mean().item() <= 3 * g_alt.mean().item() + 1e-3, (g_tp.mean().item(), g_alt.mean().item())
    # fc3 is replicated: every shard holds bitwise the same copy (same all-reduced inputs)
    for sh in shards[1:]:
        assert torch.equal(sh.layers[2].W, shards[0].layers[2].W)
    for (Wa, ba), Lr, La in zip(_full(shards), ref.layers, alt.layers):
        for a, b, c in ((Wa, Lr.W, La.W), (ba, Lr.b, La.b)):
            assert a.shape == b.shape
            d, dn = (a - b).abs(), (c - b).abs()
            assert d.max().item() <= 2 * lr * steps + 1e-6
            fd, fn = (d > 1e-4).float().mean().item(), (dn > 1e-4).float().mean().item()
            assert fd <= 3 * fn + 1e-3, (fd, fn)


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
