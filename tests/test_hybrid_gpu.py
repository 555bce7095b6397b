"""The hybrid persistent server epoch (`_C.HybridEpoch`, csrc/hybrid.hip) against fp32 PyTorch.

One launch runs a whole client epoch of Bob's SISA server training for a WIDE shard (TP = 1 /
2 / 4 of model2_sisa): fc2 / fc3 / biases and their Adam state stay on-chip, fc1 streams.
As for the register-resident epoch (tests/test_resident_gpu.py), torch cannot be
re-synchronised inside one launch, so:
* one launch per step (S = 1), torch re-synchronised before every step (weights, moments, step
  count), post-step weights / moments and losses compared (`torch.optim.Adam(lr,
  weight_decay=1e-5)`, data_entities_vanilla_sisa.py:266,305-313) on the full model2_sisa
  (fc1 5408 -> 5000, fc2 5000 -> 1000, fc3 1000 -> 100, dropout 0.5 on fc1 / fc2);
* one launch of S steps is bitwise the S one-step launches (the in-launch hand-offs and the
  prologue's look-ahead compute exactly what the launch boundaries do);
* other shard shapes (TP = 2 / 4 widths, fewer rows per step, a partial last batch through
  the launch-per-stage executor, small odd shapes) stay close to torch over free-running steps.
"""
import copy
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

from splitlearning_amd.engine import OptSlot, TailEngine, adam
from splitlearning_amd.models.zoo import LinearSpec, TailSpec, _MLP
from splitlearning_amd.ops import rng

pytestmark = pytest.mark.gpu


def _spec(n1=5000, k1=5408, n2=1000, c=100, p=0.5):
    return TailSpec([LinearSpec("fc1", k1, n1, True, p), LinearSpec("fc2", n1, n2, True, p),
                     LinearSpec("fc3", n2, c, False, 0.0)])


def _ref_forward(mod, x, seed_base, step):
    h = x
    for i, lin in enumerate(mod.linears()):
        ls = mod.spec.layers[i]
        h = F.relu(F.linear(h, lin.weight, lin.bias)) if ls.relu else F.linear(h, lin.weight, lin.bias)
        if ls.dropout:
            keep = rng.keep_mask(rng.step_seed(seed_base, i, step), h.shape[0], h.shape[1], ls.dropout,
                                 device=h.device)
            h = h * keep / (1 - ls.dropout)
    return h


def _sync_torch(ref, opt, te, slot, t):
    with torch.no_grad():
        for name, p in ref.named_parameters():
            L = te.layers[int(name[2]) - 1]
            p.copy_(L.W if name.endswith("weight") else L.b)
            st = slot.states[name]
            opt.state[p] = {"step": torch.tensor(float(t)), "exp_avg": st["m"].clone(),
                            "exp_avg_sq": st["v"].clone()}


def _engine(base, spec, cuda, seed_base, tag):
    te = TailEngine(copy.deepcopy(base), spec, cuda, seed_base=seed_base, ws_tag=tag)
    slot = OptSlot(adam(1e-3, 1e-5))
    for L in te.layers:
        slot.state(f"{L.spec.name}.weight", L.W)
        slot.state(f"{L.spec.name}.bias", L.b)
    return te, slot


def test_hybrid_step_matches_torch_adam_every_step(cuda):
    B, steps, lr, seed_base = 16, 12, 1e-3, 7
    spec = _spec()
    g = torch.Generator().manual_seed(3)
    acts = (torch.rand(B * steps, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (B * steps,), generator=g).to(cuda)
    torch.manual_seed(11)
    base = _MLP(spec)
    te, slot = _engine(base, spec, cuda, seed_base, "#hy1")
    assert te.hybrid_ok(slot, B), te._hybrid_executor(slot, B).why()
    ex = te._hybrid_executor(slot, B)
    ref = copy.deepcopy(base).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    for i in range(steps):
        x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
        _sync_torch(ref, opt, te, slot, i)
        opt.zero_grad()
        loss_r = F.cross_entropy(_ref_forward(ref, x, seed_base, i + 1), y, reduction="none")
        loss_r.mean().backward()
        opt.step()
        loss_e = torch.empty(B, device=cuda)
        fc, t, done = ex.run(x.contiguous(), y.contiguous(), loss_e, seed_base, te.fwd_count, slot.t)
        te.fwd_count, slot.t = int(fc), int(t)
        assert done == B
        torch.testing.assert_close(loss_e, loss_r.detach(), rtol=2e-4, atol=1e-4, msg=f"step {i} loss")
        for name, p in ref.named_parameters():
            L = te.layers[int(name[2]) - 1]
            e = L.W if name.endswith("weight") else L.b
            d = (e - p.detach()).abs()
            assert d.max().item() <= 2 * lr + 1e-6, (i, name, d.max().item())
            assert (d > 1e-6).float().mean().item() < 1e-4, (i, name, (d > 1e-6).float().mean().item())
            st, mine = opt.state[p], slot.states[name]
            for k, tk in (("m", "exp_avg"), ("v", "exp_avg_sq")):
                ref_k = st[tk]
                torch.testing.assert_close(mine[k], ref_k, rtol=1e-3, atol=1e-5 * ref_k.abs().max().item() + 1e-30,
                                           msg=f"step {i} {name} {k}")
    assert (te.fwd_count, slot.t) == (steps, steps)


def test_hybrid_one_launch_is_bitwise_per_step_launches(cuda):
    B, steps, seed_base = 16, 24, 5
    spec = _spec()
    g = torch.Generator().manual_seed(8)
    acts = (torch.rand(B * steps, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (B * steps,), generator=g).to(cuda)
    torch.manual_seed(12)
    base = _MLP(spec)
    one, s1 = _engine(base, spec, cuda, seed_base, "#hy2a")
    many, s2 = _engine(base, spec, cuda, seed_base, "#hy2b")
    loss_one = one.run_hybrid_epoch(acts, labels, s1, B)
    ex = many._hybrid_executor(s2, B)
    losses = []
    for i in range(steps):
        le = torch.empty(B, device=cuda)
        fc, t, _ = ex.run(acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B], le, seed_base, many.fwd_count, s2.t)
        many.fwd_count, s2.t = int(fc), int(t)
        losses.append(le)
    torch.cuda.synchronize()
    assert torch.equal(loss_one, torch.cat(losses))
    for La, Lb in zip(one.layers, many.layers):
        assert torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b)
    for k in s1.states:
        for kk in ("m", "v"):
            assert torch.equal(s1.states[k][kk], s2.states[k][kk]), (k, kk)
    assert (one.fwd_count, s1.t) == (many.fwd_count, s2.t) == (steps, steps)


@pytest.mark.parametrize("n1,n2,c,k1,B,rows", [(2500, 1000, 100, 5408, 16, 16 * 5 + 7),
                                                (1252, 1000, 100, 5408, 8, 8 * 6),
                                                (300, 256, 10, 1024, 16, 16 * 6 + 5),
                                                (160, 64, 12, 1024, 4, 4 * 9 + 3)])
def test_hybrid_shapes_free_running_close_to_torch(cuda, n1, n2, c, k1, B, rows):
    lr, seed_base = 1e-3, 2
    spec = _spec(n1=n1, n2=n2, c=c, k1=k1, p=0.25)
    g = torch.Generator().manual_seed(n1)
    acts = (torch.rand(rows, k1, generator=g) * 4).to(cuda)
    labels = torch.randint(0, c, (rows,), generator=g).to(cuda)
    torch.manual_seed(13)
    base = _MLP(spec)
    te, slot = _engine(base, spec, cuda, seed_base, f"#hy3{n1}")
    assert te.hybrid_ok(slot, B), te._hybrid_executor(slot, B).why()
    loss_e = te.run_hybrid_epoch(acts, labels, slot, B)
    ref = copy.deepcopy(base).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    losses = []
    for i, s in enumerate(range(0, rows, B)):
        x, y = acts[s:s + B], labels[s:s + B]
        opt.zero_grad()
        loss_r = F.cross_entropy(_ref_forward(ref, x, seed_base, i + 1), y, reduction="none")
        loss_r.mean().backward()
        opt.step()
        losses.append(loss_r.detach())
    torch.testing.assert_close(loss_e, torch.cat(losses), rtol=1e-3, atol=1e-3)
    for name, p in ref.named_parameters():
        L = te.layers[int(name[2]) - 1]
        e = L.W if name.endswith("weight") else L.b
        d = (e - p.detach()).abs()
        steps = -(-rows // B)
        assert d.max().item() <= 2 * lr * steps + 1e-6, (name, d.max().item())
        assert (d > 1e-4).float().mean().item() < 1e-3, (name, (d > 1e-4).float().mean().item())
    assert slot.t == -(-rows // B)


def test_hybrid_table_covers_every_tile_once(cuda):
    """The workgroups' fc1 tile runs partition the tiles in order, every row block's first
    workgroup and workgroup count match the runs, and every fc2 column block counts the fc1
    row blocks that overlap it (csrc/hybrid_exec.cpp tables)."""
    spec = _spec()
    te, slot = _engine(_MLP(spec), spec, cuda, 1, "#hy4")
    ex = te._hybrid_executor(slot, 16)
    assert ex.ok(), ex.why()
    G = ex.workgroups()
    tab = ex.table().cpu().tolist()
    nrb, ncb = (5000 + 15) // 16, (5408 + 255) // 256
    tile0 = tab[:G + 1]
    assert tile0[0] == 0 and tile0[-1] == nrb * ncb and all(b >= a for a, b in zip(tile0, tile0[1:]))
    rbw0, rbn = tab[G + 1:G + 1 + nrb], tab[G + 1 + nrb:G + 1 + 2 * nrb]
    for rb in range(nrb):
        owners = [w for w in range(G) if tile0[w] < (rb + 1) * ncb and tile0[w + 1] > rb * ncb]
        assert rbw0[rb] == owners[0] and rbn[rb] == len(owners), rb
    NC = G // 8
    hn = tab[G + 1 + 2 * nrb:]
    assert len(hn) == NC and sum(hn) >= nrb and min(hn) >= 1


@pytest.mark.parametrize("T", [2, 4, 8])
def test_hybrid_tensor_parallel_across_processes_on_one_gpu(T):
    """T = 2 / 4 real processes, each a hybrid persistent launch of 256 / T workgroups on the one
    GPU, the fc2 product exchanged through the peer-mapped region in-launch (8-byte tagged
    granules summed in rank order): replicated state and losses bitwise equal across ranks and
    close to torch (scripts/resident_tp_one_gpu.py hybrid)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "resident_tp_one_gpu.py"), str(T), "hybrid"],
                         capture_output=True, text=True, timeout=110, cwd=root)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("PASS") == T, text[-3000:]


def test_hybrid_chunked_epoch_is_bitwise_one_launch(cuda):
    """An epoch whose inputs exceed the launch's 32-bit buffer offsets runs as consecutive
    launches (csrc/hybrid_exec.cpp max_steps): forced here with chunks of 5 steps over 23 steps
    (the last chunk short), bitwise the single launch."""
    B, steps, seed_base = 16, 23, 4
    spec = _spec(n1=1252, p=0.5)
    g = torch.Generator().manual_seed(5)
    acts = (torch.rand(B * steps + 7, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (B * steps + 7,), generator=g).to(cuda)
    torch.manual_seed(14)
    base = _MLP(spec)
    one, s1 = _engine(base, spec, cuda, seed_base, "#hyc1")
    chunked, s2 = _engine(base, spec, cuda, seed_base, "#hyc2")
    chunked.hybrid_chunk_steps = 5
    assert chunked._hybrid_executor(s2, B).max_steps() == 5
    l1 = one.run_hybrid_epoch(acts, labels, s1, B)
    l2 = chunked.run_hybrid_epoch(acts, labels, s2, B)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    for La, Lb in zip(one.layers, chunked.layers):
        assert torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b)
    for k in s1.states:
        for kk in s1.states[k]:
            assert torch.equal(s1.states[k][kk], s2.states[k][kk]), (k, kk)
    assert (one.fwd_count, s1.t) == (chunked.fwd_count, s2.t) == (steps + 1, steps + 1)


def test_hybrid_sgd_momentum_close_to_torch(cuda):
    """The SGD-momentum instantiation (hybrid_epoch_kernel<false, *>: one state array, `buf`)
    against torch.optim.SGD(momentum=0.9) over free-running steps (the vanilla optimizer,
    data_entities_vanilla.py:37-42)."""
    from splitlearning_amd.engine import sgd_momentum
    B, rows, lr, seed_base = 16, 16 * 10, 1e-3, 6
    spec = _spec(n1=1252, p=0.5)
    g = torch.Generator().manual_seed(6)
    acts = (torch.rand(rows, 5408, generator=g) * 4).to(cuda)
    labels = torch.randint(0, 100, (rows,), generator=g).to(cuda)
    torch.manual_seed(15)
    base = _MLP(spec)
    te = TailEngine(copy.deepcopy(base), spec, cuda, seed_base=seed_base, ws_tag="#hysgd")
    slot = OptSlot(sgd_momentum(lr))
    for L in te.layers:
        slot.state(f"{L.spec.name}.weight", L.W)
        slot.state(f"{L.spec.name}.bias", L.b)
    assert te.hybrid_ok(slot, B), te._hybrid_executor(slot, B).why()
    loss_e = te.run_hybrid_epoch(acts, labels, slot, B)
    ref = copy.deepcopy(base).to(cuda)
    opt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9)
    losses = []
    for i, s in enumerate(range(0, rows, B)):
        x, y = acts[s:s + B], labels[s:s + B]
        opt.zero_grad()
        loss_r = F.cross_entropy(_ref_forward(ref, x, seed_base, i + 1), y, reduction="none")
        loss_r.mean().backward()
        opt.step()
        losses.append(loss_r.detach())
    torch.testing.assert_close(loss_e, torch.cat(losses), rtol=1e-3, atol=1e-3)
    for name, p in ref.named_parameters():
        L = te.layers[int(name[2]) - 1]
        e = L.W if name.endswith("weight") else L.b
        torch.testing.assert_close(e, p.detach(), rtol=1e-4, atol=1e-5, msg=name)
        torch.testing.assert_close(slot.states[name]["buf"], opt.state[p]["momentum_buffer"], rtol=1e-3,
                                   atol=1e-6 + 1e-4 * opt.state[p]["momentum_buffer"].abs().max().item(), msg=name)


def test_hybrid_mid_epoch_failure_rolls_back_to_launch_per_stage(cuda, monkeypatch):
    """`engine.resident.Failsafe` (the path SisaSession.server_epoch takes): a launch whose
    hand-off at step 5 of the second client epoch never arrives (injected: the kernel's
    fault_step) times out and raises after updating part of the shard; the shard is restored and the epoch re-runs launch-per-stage.
    The result is bitwise a job that switched executors at that epoch with no failure."""
    from splitlearning_amd.engine.resident import FAULT_EPOCH_ENV, Failsafe, _launch_per_stage_epoch
    B, rows, seed_base = 16, 16 * 12, 8
    spec = _spec(n1=1252, p=0.5)
    g = torch.Generator().manual_seed(9)
    acts = (torch.rand(rows, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (rows,), generator=g).to(cuda)
    torch.manual_seed(16)
    base = _MLP(spec)
    ta, sa = _engine(base, spec, cuda, seed_base, "#hyfa")
    ta.resident_timeout_s = 1.0          # the injected stall times out after 1 s
    tb, sb = _engine(base, spec, cuda, seed_base, "#hyfb")
    monkeypatch.setenv(FAULT_EPOCH_ENV, "0:1:5")
    fs = Failsafe(ta, sa, B)
    assert fs.run("hybrid", acts, labels)
    assert not fs.run("hybrid", acts, labels)
    assert fs.fallback["epoch"] == 1 and "error word 2" in fs.fallback["reason"]
    la = _launch_per_stage_epoch(ta, sa, acts, labels, B)
    monkeypatch.delenv(FAULT_EPOCH_ENV)
    tb.run_hybrid_epoch(acts, labels, sb, B)
    lb = _launch_per_stage_epoch(tb, sb, acts, labels, B)
    torch.cuda.synchronize()
    assert torch.equal(la, lb)
    for La, Lb in zip(ta.layers, tb.layers):
        assert torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b)
    for k in sa.states:
        for kk in sa.states[k]:
            assert torch.equal(sa.states[k][kk], sb.states[k][kk]), (k, kk)
    assert (ta.fwd_count, sa.t) == (tb.fwd_count, sb.t) == (2 * rows // B, 2 * rows // B)


@pytest.mark.parametrize("kind", ["hybrid", "resident"])
def test_tensor_parallel_mid_epoch_failure_survived_across_processes(kind):
    """T = 2 real processes on the one GPU: rank 0's persistent launch stops mid-epoch, rank 1's
    in-launch exchange times out; both ranks roll back, re-arm the peer-mapped region and finish
    on launch-per-stage; nothing raises, the state is bitwise a clean switch at that epoch and
    close to fp32 torch (scripts/persist_fallback_one_gpu.py)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "persist_fallback_one_gpu.py"), "2", kind],
                         capture_output=True, text=True, timeout=110, cwd=root)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("PASS") == 2, text[-3000:]


def test_resident_mid_epoch_failure_rolls_back_to_launch_per_stage(cuda, monkeypatch):
    """The same rollback on the register-resident executor (a TP = 8-wide shard's fc1, one
    process): a stalled hand-off at step 3 of the second epoch times out, the shard is restored
    and the epoch re-runs launch-per-stage, bitwise a clean switch at that epoch (the T = 2
    cross-process form is test_tensor_parallel_mid_epoch_failure_survived_across_processes)."""
    from splitlearning_amd.engine.resident import FAULT_EPOCH_ENV, Failsafe, _launch_per_stage_epoch
    B, rows, seed_base = 16, 16 * 10, 9
    spec = _spec(n1=628, p=0.5)
    g = torch.Generator().manual_seed(10)
    acts = (torch.rand(rows, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (rows,), generator=g).to(cuda)
    torch.manual_seed(17)
    base = _MLP(spec)
    ta, sa = _engine(base, spec, cuda, seed_base, "#rsfa")
    ta.resident_timeout_s = 1.0
    tb, sb = _engine(base, spec, cuda, seed_base, "#rsfb")
    assert ta.resident_ok(sa, B) and tb.resident_ok(sb, B)
    monkeypatch.setenv(FAULT_EPOCH_ENV, "0:1:3")
    fs = Failsafe(ta, sa, B)
    assert fs.run("resident", acts, labels)
    assert not fs.run("resident", acts, labels)
    assert fs.fallback["epoch"] == 1 and "error word 2" in fs.fallback["reason"]
    la = _launch_per_stage_epoch(ta, sa, acts, labels, B)
    monkeypatch.delenv(FAULT_EPOCH_ENV)
    tb.run_resident_epoch(acts, labels, sb, B)
    lb = _launch_per_stage_epoch(tb, sb, acts, labels, B)
    torch.cuda.synchronize()
    assert torch.equal(la, lb)
    for La, Lb in zip(ta.layers, tb.layers):
        assert torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b)
    for k in sa.states:
        for kk in sa.states[k]:
            assert torch.equal(sa.states[k][kk], sb.states[k][kk]), (k, kk)


@pytest.mark.parametrize("kind,n1", [("hybrid", 1252), ("resident", 628)])
def test_whole_server_epoch_with_short_batches_in_one_launch(cuda, kind, n1):
    """One server epoch over three clients' caches with short final batches (50, 37, 64 rows at
    B = 16) as ONE persistent call (`TailEngine.padded_plan`: every short batch zero-padded
    with ignored labels, its CE mean over its real rows).  Every step of the plan, launched on
    its own from torch's synced state, matches torch replaying the reference loop
    `for cid: for batch in cid's cached batches: step` (data_entities_vanilla_sisa.py:298-313)
    on the batch's real rows; and the whole plan in one call is bitwise those per-step launches
    (an unsynced 11-step Adam comparison would only measure how fast fp32 rounding amplifies)."""
    B, lr, seed_base = 16, 1e-3, 3
    spec = _spec(n1=n1, p=0.5)
    g = torch.Generator().manual_seed(11)
    caches = []
    for n in (50, 37, 64):
        caches.append(((torch.rand(n, 5408, generator=g) * 20).to(cuda), torch.randint(0, 100, (n,), generator=g).to(cuda)))
    torch.manual_seed(18)
    base = _MLP(spec)
    X, Y, rows = TailEngine.padded_plan(caches, B)
    assert rows == [16, 16, 16, 2, 16, 16, 5, 16, 16, 16, 16] and X.shape[0] == 16 * len(rows)
    # per step, each from torch's synced state
    te, slot = _engine(base, spec, cuda, seed_base, f"#plan{kind}a")
    assert (te.resident_ok(slot, B) if kind == "resident" else te.hybrid_ok(slot, B))
    ex = te._resident_executor(slot, B) if kind == "resident" else te._hybrid_executor(slot, B)
    ref = copy.deepcopy(base).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    per_step = []
    for i, r in enumerate(rows):
        x, y = X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B]
        assert torch.all(y[r:] == -100) and torch.all(x[r:] == 0)
        _sync_torch(ref, opt, te, slot, i)
        opt.zero_grad()
        loss_r = F.cross_entropy(_ref_forward(ref, x[:r], seed_base, i + 1), y[:r], reduction="none")
        loss_r.mean().backward()
        opt.step()
        loss_e = torch.empty(B, device=cuda)
        fc, t, done = ex.run(x.contiguous(), y.contiguous(), loss_e, seed_base, te.fwd_count, slot.t, step_rows=[r])
        te.fwd_count, slot.t = int(fc), int(t)
        assert done == B
        per_step.append(loss_e)
        assert torch.all(loss_e[r:] == 0), "padded rows carry no loss"
        torch.testing.assert_close(loss_e[:r], loss_r.detach(), rtol=2e-4, atol=1e-4, msg=f"step {i} loss")
        for name, p in ref.named_parameters():
            L = te.layers[int(name[2]) - 1]
            e = L.W if name.endswith("weight") else L.b
            d = (e - p.detach()).abs()
            assert d.max().item() <= 2 * lr + 1e-6, (i, name, d.max().item())
            # Adam's first steps move a near-zero-gradient entry by about +-lr whichever way its
            # fp32 gradient rounds: a few such entries per tensor, however small the tensor
            assert (d > 1e-6).sum().item() <= max(2, 1e-4 * d.numel()), (i, name, (d > 1e-6).sum().item())
    # the whole plan in one call
    tw, sw = _engine(base, spec, cuda, seed_base, f"#plan{kind}b")
    run = tw.run_resident_epoch if kind == "resident" else tw.run_hybrid_epoch
    loss = run(X, Y, sw, B, rows)
    torch.cuda.synchronize()
    assert (tw.fwd_count, sw.t) == (len(rows), len(rows))
    assert torch.equal(loss, torch.cat(per_step))
    for La, Lb in zip(te.layers, tw.layers):
        assert torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b)


@pytest.mark.parametrize("kind,n1", [("hybrid", 1252), ("resident", 628)])
def test_nonfinite_epoch_rolls_back(cuda, kind, n1):
    """A NaN injected into one epoch's inputs: the launch finishes, but its losses and shard are
    non-finite; `Failsafe` restores the pre-epoch shard (bitwise) and reports the fallback, so
    the caller re-runs that epoch launch-per-stage instead of training on garbage."""
    from splitlearning_amd.engine.resident import Failsafe
    B, rows, seed_base = 16, 16 * 6, 4
    spec = _spec(n1=n1, p=0.5)
    g = torch.Generator().manual_seed(12)
    acts = (torch.rand(rows, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (rows,), generator=g).to(cuda)
    torch.manual_seed(19)
    base = _MLP(spec)
    te, slot = _engine(base, spec, cuda, seed_base, f"#nan{kind}")
    assert te.resident_ok(slot, B) if kind == "resident" else te.hybrid_ok(slot, B)
    fs = Failsafe(te, slot, B)
    assert fs.run(kind, acts, labels)                       # a clean epoch is kept
    before = [L.W.clone() for L in te.layers] + [v.clone() for st in slot.states.values() for v in st.values()]
    counters = (te.fwd_count, slot.t)
    bad = acts.clone()
    bad[3 * B + 5, 100] = float("nan")                      # one element of step 3's batch
    assert not fs.run(kind, bad, labels)
    assert fs.fallback["epoch"] == 1 and "non-finite" in fs.fallback["reason"], fs.fallback
    after = [L.W for L in te.layers] + [v for st in slot.states.values() for v in st.values()]
    assert all(torch.equal(x, y) for x, y in zip(before, after))
    assert (te.fwd_count, slot.t) == counters
