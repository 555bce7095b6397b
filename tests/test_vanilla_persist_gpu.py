"""Vanilla persistent split epoch (`_C.VanillaEpoch`, csrc/vanilla.hip): a co-located Alice's
whole vanilla epoch -- her conv front and Bob's 3-layer tail, forward, CE, backward and both
SGD-momentum steps, a short final batch included -- in ONE launch.

Checked against the per-batch native executor (csrc/split.cpp), itself bitwise the Python loop
(tests/test_split_native_gpu.py) whose kernels are torch-checked: every parameter, momentum
buffer, step count and dropout counter after two epochs and an unlearn-style restart agree to
fp32 rounding (the kernel sums in its own fixed order).  One launch of S steps is bitwise S
one-step launches, and a launch that fails mid-epoch falls back, restored, to the per-batch
executor with bitwise that executor's result.  Reference hot loop: data_entities_vanilla.py:66-76."""
import pytest
import torch

from test_split_native_gpu import _session, _states

pytestmark = pytest.mark.gpu


def _close(a, b, what):
    assert a.keys() == b.keys()
    for k in a:
        x, y = a[k], b[k]
        scale = max(float(y.abs().max()), 1e-6)
        torch.testing.assert_close(x, y, rtol=1e-4, atol=2e-5 * scale, msg=f"{what}: {k}")


def _epochs(s, order, B):
    for _ in range(2):
        s.split_epoch(1, order, order.numel())
    s.alices[1].slot = type(s.alices[1].slot)(s.alice_optim())
    s.bob_slots[1] = type(s.bob_slots[1])(s.bob_optim())
    s.split_epoch(1, order[: B * 3], B * 3)


@pytest.mark.parametrize("B", [16, 5])
def test_persistent_vanilla_matches_per_batch(cuda, tmp_path, B):
    from splitlearning_amd.protocols.split_native import persistent_vanilla_ok
    sp = _session("vanilla", tmp_path, True, cuda, B)
    sq = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    assert persistent_vanilla_ok(sq, 1) and not persistent_vanilla_ok(sp, 1)
    order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(4))[:B * 6 + 3].to(cuda)
    for s in (sp, sq):
        _epochs(s, order, B)
    torch.cuda.synchronize()
    assert sq.native_split_epochs.get("persistent") == 3, (sq.native_split_epochs, sq.__dict__.get("split_persist_reason"))
    _close(_states(sq, "vanilla"), _states(sp, "vanilla"), f"B={B}")
    assert sp.alices[1].slot.t == sq.alices[1].slot.t and sp.bob_slot(1).t == sq.bob_slot(1).t
    assert sp.tail.fwd_count == sq.tail.fwd_count


def test_persistent_vanilla_one_launch_is_bitwise_step_launches(cuda, tmp_path):
    B = 16
    s1 = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    s2 = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    s3 = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    s3._va_max_steps = 2          # the executor's own chunking: launches of at most 2 steps
    order = s1.alices[1].train.shuffled_order(torch.Generator().manual_seed(7))[:B * 5 + 7].to(cuda)
    s1.split_epoch(1, order, order.numel())
    s3.split_epoch(1, order, order.numel())
    for i in range(0, order.numel(), B):
        part = order[i:i + B]
        s2.split_epoch(1, part, part.numel())
    torch.cuda.synchronize()
    assert s1.native_split_epochs["persistent"] == 1 and s2.native_split_epochs["persistent"] == 6
    a, b, c = _states(s1, "vanilla"), _states(s2, "vanilla"), _states(s3, "vanilla")
    for k in a:
        assert torch.equal(a[k], b[k]), k
        assert torch.equal(a[k], c[k]), k
    assert s1.tail.fwd_count == s2.tail.fwd_count and s1.bob_slot(1).t == s2.bob_slot(1).t


def test_persistent_vanilla_mid_epoch_failure_falls_back(cuda, tmp_path):
    """A hand-off that never arrives at step 3: the launch gives up, the snapshot is restored
    and the epoch reruns on the per-batch executor -- bitwise a run that never tried."""
    B = 16
    sp = _session("vanilla", tmp_path, True, cuda, B)
    sq = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    sq.args.persist_timeout_s = 0.5
    order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(5))[:B * 6].to(cuda)
    sq._va_fault_step = 3
    for s in (sp, sq):
        s.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    assert "persistent" not in sq.native_split_epochs and sq.split_persist_fallback
    a, b = _states(sq, "vanilla"), _states(sp, "vanilla")
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_persistent_vanilla_update_runs_partition_the_tiles(cuda, tmp_path):
    """The update-pass table (csrc/vanilla_exec.cpp tables): the G balanced column-major runs
    partition fc1's tiles, each column block counts the runs touching it and numbers them in run
    order (the dx partials' sum order, as when runs were dealt in order), and the runs are dealt
    to workgroups by the row band they start in (workgroup w on XCD w % 8 stages ~1/4 of the row
    blocks' dz1, not all of them)."""
    from splitlearning_amd.protocols.split_native import _va_cfg
    s = _session("vanilla", tmp_path, True, cuda, 16, persist=True)
    ex = s.ops.C().VanillaEpoch(_va_cfg(s, 1))
    assert ex.ok(), ex.why()
    G = ex.workgroups()
    tab = ex.table().cpu().tolist()
    N1, K1 = s.tail.layers[0].W.shape
    nrb, ncb, NC = (N1 + 15) // 16, (K1 + 255) // 256, G // 8
    oU = G + 1 + 2 * nrb + NC
    oUW, oUS = oU + ncb, oU + ncb + 4 * G
    assert len(tab) == oUS + G * ncb
    cbn = tab[oU:oU + ncb]
    runs = [tab[oUW + 4 * w:oUW + 4 * w + 4] for w in range(G)]
    assert all(r[2] == 0 and r[3] == nrb for r in runs)
    T = nrb * ncb
    assert sorted((r[0], r[1]) for r in runs) == [(k * T // G, (k + 1) * T // G) for k in range(G)]
    seen = [0] * ncb
    for v0, v1, _, _ in sorted(runs):
        w = next(x for x in range(G) if runs[x][0] == v0 and runs[x][1] == v1)
        for cb in range(ncb):
            slot = tab[oUS + w * ncb + cb]
            touches = v1 > v0 and v0 // nrb <= cb <= (v1 - 1) // nrb
            assert (slot >= 0) == touches, (w, cb)
            if touches:
                assert slot == seen[cb], (w, cb)
                seen[cb] += 1
    assert seen == cbn
    if G % 8 == 0 and nrb >= 64:
        home = sum(1 for w in range(G) if (runs[w][0] % nrb) * 8 // nrb == w % 8)
        assert home >= G - G // 16, home
