"""The register-resident server epoch (`_C.ResidentEpoch`, csrc/resident.hip) against fp32
PyTorch.

The persistent launch keeps a narrow shard's weights and Adam state on-chip for all of its
steps, so torch cannot be re-synchronised inside one launch.  Three checks instead:
* one launch per step (S = 1), torch re-synchronised before every step (weights, moments,
  step count), post-step weights / moments and losses compared, as tests/test_golden_gpu.py
  does for the launch-per-stage executor (`torch.optim.Adam(lr, weight_decay=1e-5)`,
  data_entities_vanilla_sisa.py:266,305-313), on a TP = 8 shard shape of model2_sisa
  (fc1 5408 -> 625, fc2 625 -> 1000, fc3 1000 -> 100, dropout 0.5 on fc1 / fc2);
* one launch of S steps is bitwise the S one-step launches (the in-launch hand-offs and the
  prologue's look-ahead compute exactly what the launch boundaries do);
* odd shapes (an fc1 shard that is not a multiple of 16 rows, fewer rows per step, a partial
  last batch through the launch-per-stage executor) stay close to torch over a few
  free-running steps.
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _spec(n1=625, k1=5408, n2=1000, c=100, p=0.5):
    return TailSpec([LinearSpec("fc1", k1, n1, True, p), LinearSpec("fc2", n1, n2, True, p),
                     LinearSpec("fc3", n2, c, False, 0.0)])


def _ref_forward(mod, x, seed_base, step, col_off=0):
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


def test_resident_step_matches_torch_adam_every_step(cuda):
    B, steps, lr, seed_base = 16, 24, 1e-3, 7
    spec = _spec()
    g = torch.Generator().manual_seed(3)
    acts = (torch.rand(B * steps, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (B * steps,), generator=g).to(cuda)
    torch.manual_seed(11)
    base = _MLP(spec)
    te, slot = _engine(base, spec, cuda, seed_base, "#res1")
    assert te.resident_ok(slot, B), te._resident_executor(slot, B).why()
    ex = te._resident_executor(slot, B)
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


def test_resident_one_launch_is_bitwise_per_step_launches(cuda):
    B, steps, seed_base = 16, 40, 5
    spec = _spec()
    g = torch.Generator().manual_seed(8)
    acts = (torch.rand(B * steps, 5408, generator=g) * 20).to(cuda)
    labels = torch.randint(0, 100, (B * steps,), generator=g).to(cuda)
    torch.manual_seed(12)
    base = _MLP(spec)
    one, s1 = _engine(base, spec, cuda, seed_base, "#res2a")
    many, s2 = _engine(base, spec, cuda, seed_base, "#res2b")
    loss_one = one.run_resident_epoch(acts, labels, s1, B)
    ex = many._resident_executor(s2, B)
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


@pytest.mark.parametrize("n1,n2,c,B,rows", [(300, 256, 10, 16, 16 * 6 + 5), (625, 1000, 100, 8, 8 * 7),
                                             (36, 64, 12, 4, 4 * 9 + 3)])
def test_resident_odd_shapes_free_running_close_to_torch(cuda, n1, n2, c, B, rows):
    lr, seed_base = 1e-3, 2
    spec = _spec(n1=n1, n2=n2, c=c, k1=1024, p=0.25)
    g = torch.Generator().manual_seed(n1)
    acts = (torch.rand(rows, 1024, generator=g) * 4).to(cuda)
    labels = torch.randint(0, c, (rows,), generator=g).to(cuda)
    torch.manual_seed(13)
    base = _MLP(spec)
    te, slot = _engine(base, spec, cuda, seed_base, f"#res3{n1}")
    assert te.resident_ok(slot, B), te._resident_executor(slot, B).why()
    loss_e = te.run_resident_epoch(acts, labels, slot, B)
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


def test_resident_rejects_a_wide_shard(cuda):
    from splitlearning_amd.models import ServerTailSisa, sisa_server_spec
    te = TailEngine(ServerTailSisa(), sisa_server_spec(), cuda, ws_tag="#res4")
    slot = OptSlot(adam(1e-3, 1e-5))
    assert not te.resident_ok(slot, 16)          # fc1 5000 rows: the launch-per-stage executor


@pytest.mark.parametrize("T", [2, 4, 8])
def test_resident_tensor_parallel_across_processes_on_one_gpu(T):
    """T = 2 / 4 / 8 real processes, each a persistent launch of 256 / T workgroups on the one GPU
    (T = 8: the multi-GPU granule protocol at its production width, on a scaled-down tail),
    the fc2 exchange through the peer-mapped region in-launch (T-source granule sums): replicated
    state and losses bitwise equal across ranks and close to torch
    (scripts/resident_tp_one_gpu.py)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "resident_tp_one_gpu.py"), str(T)],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("PASS") == T, text[-3000:]


def test_probe_adopts_resident_executor_across_processes():
    """engine/resident.py decide at T = 2 real processes: both probes pass with the same fc3,
    both ranks adopt the resident executor and train an epoch on it."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "resident_probe_fault_one_gpu.py"), "2", "-1"],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("adopted True") == 2 and out.stdout.count("PASS") == 2, text[-3000:]


def test_failed_probe_falls_back_on_every_rank():
    """A probe exchange timeout on one rank (rank 1 skips its probe launch, so rank 0's in-launch
    exchange times out and raises the peer-mapped region's error word): every rank agrees not to
    adopt, the region is re-armed on every rank (error word clear), and both ranks then train a
    server epoch on the launch-per-stage executor's fused peer-mapped all-reduce with the
    replicated fc3 bitwise equal; nothing raises (reference split_nn.py:183-186)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "resident_probe_fault_one_gpu.py"), "2", "1"],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("adopted False") == 2, text[-3000:]
    assert out.stdout.count("launch-per-stage executor finished, error word 0") == 2, text[-3000:]
    assert out.stdout.count("PASS") == 2, text[-3000:]


def test_sisa_session_runs_its_server_epochs_on_the_resident_executor(cuda, tmp_path):
    """The production SISA protocol (local training -> frozen-front dump -> server epochs) with a
    Bob tail as narrow as a TP = 8 shard (fc1 5408 -> 628): `_decide_resident` adopts the
    resident executor, every server epoch runs on it (the launch-per-stage executor only gets
    the trailing partial batch), and its result is held to the golden standard: an fp32 torch
    replay of the same server epoch (same cached activations, batch order, dropout seeds,
    torch.optim.Adam(lr, weight_decay=1e-5), data_entities_vanilla_sisa.py:266,298-313) is
    compared with both executors.  The resident run may not diverge from torch more than the
    launch-per-stage executor does (free-running fp32 runs in different summation orders
    drift apart under Adam's normalised steps, so the launch-per-stage executor's own
    divergence is the yardstick)."""
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import SisaSession
    from splitlearning_amd.protocols.schedule import build_steps

    spec = _spec(n1=628)

    class Narrow(SisaSession):
        def bob_module_and_spec(self):   # a TP = 8 shard's width (shards are multiples of 4 wide)
            return self.make_bob_module(_MLP, spec), spec

    runs = {}
    for res in ("auto", "off"):
        args = parse_args(["--sisa", "--world_size", "2", "--seed", "5", "--num_samples", "1400", "--no_tqdm",
                           "--server_epochs", "1", "--resident", res, "--hybrid", res,
                           "--datapath", str(tmp_path / f"d{res}"), "--log_dir", str(tmp_path / f"l{res}")])
        write_shards(args, verbose=False)
        sess = Narrow(args, Comm(0, 1, cuda, Placement.make(2, 1, 1)), cuda)
        assert sess._resident_ok == (res == "auto")
        assert sess.resident_status["adopted"] == (res == "auto")
        calls = {"native": 0}
        orig = sess.tail.run_native_epoch

        def counted(*a, **k):
            calls["native"] += 1
            return orig(*a, **k)
        sess.tail.run_native_epoch = counted
        steps = dict(build_steps(sess, args))
        steps["local_training"]()
        init = [(L.W.clone(), L.b.clone()) for L in sess.tail.layers]
        assert sess.tail.fwd_count == 0
        steps["server_training"]()
        torch.cuda.synchronize()
        runs[res] = (sess, calls["native"], init)
    sa, na, init = runs["auto"]
    so, no, init_o = runs["off"]
    n_train = sum(sa.n_train.values())
    assert sa.bob_slot.t == so.bob_slot.t == -(-n_train // 16)
    # the resident run issues the trailing partial batch (if any) on the launch-per-stage executor only
    assert na <= 1 and no >= 1
    for (wa, ba), (wo, bo) in zip(init, init_o):
        assert torch.equal(wa, wo) and torch.equal(ba, bo)
    # the torch replay of the server epoch
    acts, labels = sa.activation_and_labels_cache[(1, False, None)]
    acts = acts.float()
    ref = _MLP(spec).to(cuda)
    with torch.no_grad():
        for lin, (w, b) in zip(ref.linears(), init):
            lin.weight.copy_(w)
            lin.bias.copy_(b)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
    B = 16
    for i, s0 in enumerate(range(0, labels.numel(), B)):
        opt.zero_grad()
        F.cross_entropy(_ref_forward(ref, acts[s0:s0 + B], sa.tail.seed_base, i + 1), labels[s0:s0 + B]).backward()
        opt.step()
    for li, lin in enumerate(ref.linears()):
        for pa, po, pr, nm in ((sa.tail.layers[li].W, so.tail.layers[li].W, lin.weight, "W"),
                               (sa.tail.layers[li].b, so.tail.layers[li].b, lin.bias, "b")):
            assert torch.isfinite(pa).all()
            d_res = (pa - pr.detach()).abs()
            d_lps = (po - pr.detach()).abs()
            f_res = (d_res > 1e-4).float().mean().item()
            f_lps = (d_lps > 1e-4).float().mean().item()
            print(f"fc{li + 1}.{nm}: resident vs torch frac>1e-4 {f_res:.4f} mean {d_res.mean().item():.2e}; "
                  f"launch-per-stage vs torch {f_lps:.4f} mean {d_lps.mean().item():.2e}")
            assert d_res.max().item() <= 2 * 1e-3 * sa.bob_slot.t + 1e-6
            assert f_res <= 1.5 * f_lps + 1e-3, (li, nm, f_res, f_lps)
            assert d_res.mean().item() <= 1.5 * d_lps.mean().item() + 1e-7, (li, nm, d_res.mean().item(),
                                                                              d_lps.mean().item())
