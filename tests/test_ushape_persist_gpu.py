"""U-shape persistent split epoch (`_C.UShapeEpoch`, csrc/ushape.hip): a co-located Alice's
whole U-shape epoch -- her conv front (model1) and head (model3), Bob's model2, the CE, both
backwards and every Adam step -- in ONE launch with every parameter and moment on-chip.

Torch per step: tests/test_golden_modes_gpu.py::test_ushape_split_epoch_matches_composed_torch_adam_every_step
runs every batch through this kernel as a one-step launch, re-synchronised with one torch Adam
over model1 + model2 + model3 before each batch.  Here: several epochs (short final batches
included) and an unlearn-style restart agree with the per-batch executor (itself torch-checked)
within the Adam bound; one launch is bitwise S one-step launches and bitwise the executor's own
chunked launches; a hand-off that never arrives falls back, restored, to the per-batch executor
with bitwise its result; and a 1,000-step launch is bitwise ten 100-step launches.
Reference hot loop: data_entities.py:65-81."""
import pytest
import torch

from test_split_native_gpu import _session, _states

from splitlearning_amd.config import parse_args
from splitlearning_amd.data.mnist import write_shards
from splitlearning_amd.parallel.dist import Comm, Placement

pytestmark = pytest.mark.gpu


def _close_adam(a, b, lr, steps, what, frac=2e-3, tol=1e-4):
    assert a.keys() == b.keys()
    for k in a:
        d = (a[k].float() - b[k].float()).abs()
        if k.endswith((".m", ".v")):
            scale = max(float(b[k].abs().max()), 1e-12)
            assert d.max().item() <= 0.05 * scale + 1e-8, (what, k, d.max().item(), scale)
            continue
        assert d.max().item() <= 2 * lr * steps + 1e-6, (what, k, d.max().item())
        assert (d > tol).float().mean().item() < frac, (what, k, (d > tol).float().mean().item())


def _epochs(s, order, B):
    for _ in range(2):
        s.split_epoch(1, order, order.numel())
    s.alices[1].slot = type(s.alices[1].slot)(s.alice_optim())
    s.bob_slots[1] = type(s.bob_slots[1])(s.bob_optim())
    s.split_epoch(1, order[: B * 3], B * 3)


@pytest.mark.parametrize("B", [16, 5])
def test_persistent_ushape_matches_per_batch(cuda, tmp_path, B):
    from splitlearning_amd.protocols.split_native import persistent_ushape_ok
    sp = _session("ushape", tmp_path, True, cuda, B)
    sq = _session("ushape", tmp_path, True, cuda, B, persist=True)
    assert persistent_ushape_ok(sq, 1) and not persistent_ushape_ok(sp, 1)
    order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(4))[:B * 6 + 3].to(cuda)
    for s in (sp, sq):
        _epochs(s, order, B)
    torch.cuda.synchronize()
    assert sq.native_split_epochs.get("persistent") == 3, (sq.native_split_epochs, sq.__dict__.get("split_persist_reason"),
                                                           sq.__dict__.get("split_persist_fallback"))
    _close_adam(_states(sq, "ushape"), _states(sp, "ushape"), sq.args.lr, 2 * 7 + 3, f"B={B}")
    assert sp.alices[1].slot.t == sq.alices[1].slot.t and sp.bob_slot(1).t == sq.bob_slot(1).t
    assert sp.tail.fwd_count == sq.tail.fwd_count and sp.alices[1].head.fwd_count == sq.alices[1].head.fwd_count


def test_persistent_ushape_one_launch_is_bitwise_step_launches(cuda, tmp_path):
    B = 16
    s1 = _session("ushape", tmp_path, True, cuda, B, persist=True)
    s2 = _session("ushape", tmp_path, True, cuda, B, persist=True)
    s3 = _session("ushape", tmp_path, True, cuda, B, persist=True)
    s3._us_max_steps = 2          # the executor's own chunking: launches of at most 2 steps
    order = s1.alices[1].train.shuffled_order(torch.Generator().manual_seed(7))[:B * 5 + 7].to(cuda)
    s1.split_epoch(1, order, order.numel())
    s3.split_epoch(1, order, order.numel())
    for i in range(0, order.numel(), B):
        part = order[i:i + B]
        s2.split_epoch(1, part, part.numel())
    torch.cuda.synchronize()
    assert s1.native_split_epochs["persistent"] == 1 and s2.native_split_epochs["persistent"] == 6
    a, b, c = _states(s1, "ushape"), _states(s2, "ushape"), _states(s3, "ushape")
    for k in a:
        assert torch.equal(a[k], b[k]), k
        assert torch.equal(a[k], c[k]), k
    assert torch.equal(s1.last_split_losses, s3.last_split_losses)


def test_persistent_ushape_mid_epoch_failure_falls_back(cuda, tmp_path):
    """A hand-off that never arrives at step 3: the launch gives up, the snapshot is restored
    and the epoch reruns on the per-batch executor -- bitwise a run that never tried."""
    B = 16
    sp = _session("ushape", tmp_path, True, cuda, B)
    sq = _session("ushape", tmp_path, True, cuda, B, persist=True)
    sq.args.persist_timeout_s = 0.5
    order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(5))[:B * 6].to(cuda)
    sq._us_fault_step = 3
    for s in (sp, sq):
        s.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    assert "persistent" not in sq.native_split_epochs and sq.split_persist_fallback
    a, b = _states(sq, "ushape"), _states(sp, "ushape")
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_persistent_ushape_long_launch_is_bitwise_chunks(cuda, tmp_path):
    """1,000 steps + a short one in ONE launch, bitwise ten 100-step launches; finite."""
    B, steps = 16, 1000
    s1 = _session("ushape", tmp_path, True, cuda, B, persist=True)
    s2 = _session("ushape", tmp_path, True, cuda, B, persist=True)
    s2._us_max_steps = 100
    tr = s1.alices[1].train
    reps = -(-(steps * B + 7) // len(tr.y))
    order = torch.cat([tr.shuffled_order(torch.Generator().manual_seed(60 + r)) for r in range(reps)])
    order = order[:steps * B + 7].to(cuda)
    for s in (s1, s2):
        s.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    assert s1.native_split_epochs.get("persistent") == 1 and s2.native_split_epochs.get("persistent") == 1
    a, b = _states(s1, "ushape"), _states(s2, "ushape")
    for k in a:
        assert torch.equal(a[k], b[k]), k
        assert torch.isfinite(a[k]).all(), k
    assert torch.equal(s1.last_split_losses, s2.last_split_losses)


def _session_bf16(tmp_path, dev, persist, B=16):
    """A U-shape session under --dtype bf16 (the per-batch kernels and the persistent kernel's
    bf16 instantiation: bf16 operands, fp32 accumulation, state and moments)."""
    from splitlearning_amd.protocols import UShapeSession
    flags = ["--dtype", "bf16"] + ([] if persist else ["--split_persist", "off"])
    args = parse_args(flags + ["--world_size", "2", "--seed", "11", "--num_samples", "900", "--no_tqdm",
                               "--batch_size", str(B), "--datapath", str(tmp_path / "d"),
                               "--log_dir", str(tmp_path / "logs_bf")])
    if not (tmp_path / "d").exists():
        write_shards(args, verbose=False)
    return UShapeSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)


def test_persistent_ushape_bf16_matches_per_batch_bf16(cuda, tmp_path):
    """--dtype bf16: the persistent epoch runs (bf16 instantiation), agrees with the per-batch
    bf16 executor within the Adam bound, differs from the fp32 persistent epoch (the bf16
    products really ran), and one launch is bitwise its one-step launches."""
    from splitlearning_amd.ops import hip_ops
    from splitlearning_amd.protocols.split_native import persistent_ushape_ok
    B = 16
    try:
        sp = _session_bf16(tmp_path, cuda, False)
        sq = _session_bf16(tmp_path, cuda, True)
        s1 = _session_bf16(tmp_path, cuda, True)
        assert hip_ops.C().get_compute_dtype() == "bf16"
        assert persistent_ushape_ok(sq, 1) and not persistent_ushape_ok(sp, 1)
        order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(4))[:B * 6 + 3].to(cuda)
        for s in (sp, sq):
            _epochs(s, order, B)
        for i in range(0, order.numel(), B):
            part = order[i:i + B]
            s1.split_epoch(1, part, part.numel())
        torch.cuda.synchronize()
        assert sq.native_split_epochs.get("persistent") == 3, (sq.__dict__.get("split_persist_reason"),
                                                               sq.__dict__.get("split_persist_fallback"))
        _close_adam(_states(sq, "ushape"), _states(sp, "ushape"), sq.args.lr, 2 * 7 + 3, "bf16", frac=2e-2)
        # one launch (the first epoch of sq) vs one-step launches: replay the first epoch alone
        s2 = _session_bf16(tmp_path, cuda, True)
        s2.split_epoch(1, order, order.numel())
        torch.cuda.synchronize()
        a, b = _states(s2, "ushape"), _states(s1, "ushape")
        for k in a:
            assert torch.equal(a[k], b[k]), k
    finally:
        hip_ops.C().set_compute_dtype("fp32")
    sf = _session("ushape", tmp_path, True, cuda, B, persist=True)
    sf.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    f = _states(sf, "ushape")
    assert any(not torch.equal(f[k], a[k]) for k in a if k.endswith(".W"))
