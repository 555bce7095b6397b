"""Long persistent launches: 1,000+ steps in ONE launch of each persistent executor.

The short-launch tests (tests/test_hybrid_gpu.py, test_resident_gpu.py,
test_vanilla_persist_gpu.py) run <= 41 steps per launch; the bench runs launches of thousands
of steps.  Here, for the hybrid (csrc/hybrid.hip), register-resident (csrc/resident.hip) and
vanilla (csrc/vanilla.hip) epochs:
* one launch of >= 1,000 steps is BITWISE the same steps as ten 100-step launches (every
  in-launch hand-off of a long launch computes exactly what a launch boundary does: a stale
  or torn hand-off anywhere in the long launch would show here);
* the long launch stays within fp32 tolerance of the launch-per-stage / per-batch executor
  (a different summation order, so not bitwise).  Over 1,000 free-running steps with dropout
  and ReLU masks any fp32 rounding difference grows (a flipped mask changes a gradient), so the
  tolerance is calibrated in the same test: a CONTROL run of the reference executor on inputs
  perturbed by one ulp gives the divergence fp32 rounding alone produces, and the persistent
  executor's distance from the reference must stay within a small multiple of it for every
  parameter and for the losses.  A wrong hand-off is far outside.  (The optimizer moments are
  not compared free-running: on this random-label data most fc1 units die within ~500 steps,
  every moment of a dead unit decays towards 0, and whether a unit near the edge is dead or
  alive at step 1,000 is decided by rounding -- one surviving 16-row block dominated the
  relative distance of fc1's first moment at 4.6 x while the weights agreed to the control's
  level.  Synced to torch before every step, the hybrid's fc1 moments match to 1e-6 of their
  scale over all 1,000 steps: scripts/probe/synced_drift.py, profiles/r6_long_launch/.)
Reference loops: data_entities_vanilla_sisa.py:298-313 (server epoch), data_entities_vanilla.py:66-76
(vanilla epoch)."""
import pytest
import torch

from splitlearning_amd.engine.resident import _launch_per_stage_epoch
from splitlearning_amd.models.zoo import _MLP
from test_hybrid_gpu import _engine, _spec
from test_split_native_gpu import _session, _states

pytestmark = pytest.mark.gpu

STEPS, CHUNK = 1000, 100
# the persistent executor's distance from the reference executor may be this multiple of the
# one-ulp control's distance (different summation orders are a rounding-sized perturbation)
FACTOR = 8.0


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _ulp(x):
    """x with every element moved by at most one ulp (a rounding-sized perturbation)."""
    bits = x.contiguous().view(torch.int32)
    g = torch.Generator(device=x.device).manual_seed(99)
    step = torch.randint(-1, 2, bits.shape, generator=g, device=x.device, dtype=torch.int32)
    return (bits + step * (x != 0).to(torch.int32)).view(torch.float32)


def _check_close(name, test, ref, ctl, lt, lr, lc):
    """Every tensor of `test` within FACTOR x the control's rounding divergence from `ref`."""
    rows = []
    for k in ref:
        if k.endswith((".m", ".v", ".buf")) or ".s0" in k:
            continue                      # optimizer moments: see the module docstring
        d, c = _rel(test[k], ref[k]), _rel(ctl[k], ref[k])
        rows.append((d / max(c, 1e-7), d, c, k))
    gap_t = (lt[-CHUNK * 16:] - lr[-CHUNK * 16:]).abs().mean().item()
    gap_c = (lc[-CHUNK * 16:] - lr[-CHUNK * 16:]).abs().mean().item()
    worst = max(rows)
    print(f"{name}: worst tensor {worst[3]}: rel L2 vs reference {worst[1]:.3g}, one-ulp control {worst[2]:.3g}; "
          f"last-100-step mean loss gap {gap_t:.3g} (control {gap_c:.3g})")
    for r in sorted(rows, reverse=True)[:6]:
        print(f"   {r[3]:24s} test {r[1]:.3g} control {r[2]:.3g}")
    assert all(d <= FACTOR * c + 1e-6 for _, d, c, _ in rows), worst
    assert gap_t <= FACTOR * gap_c + 1e-6, (gap_t, gap_c)


def _tail_states(te, slot):
    out = {}
    for L in te.layers:
        out[f"{L.spec.name}.W"], out[f"{L.spec.name}.b"] = L.W, L.b
    for k, st in slot.states.items():
        for kk, v in st.items():
            out[f"{k}.{kk}"] = v
    return out


@pytest.mark.parametrize("kind,n1", [("hybrid", 5000), ("resident", 628)])
def test_server_epoch_long_launch(cuda, kind, n1):
    B, seed_base = 16, 21
    spec = _spec(n1=n1, p=0.5)
    g = torch.Generator(device=cuda).manual_seed(5)
    acts = torch.rand(B * STEPS, 5408, generator=g, device=cuda) * 20
    labels = torch.randint(0, 100, (B * STEPS,), generator=g, device=cuda)
    torch.manual_seed(23)
    base = _MLP(spec)
    one, s1 = _engine(base, spec, cuda, seed_base, f"#long{kind}1")
    chunked, s2 = _engine(base, spec, cuda, seed_base, f"#long{kind}2")
    lps, s3 = _engine(base, spec, cuda, seed_base, f"#long{kind}3")
    ctl, s4 = _engine(base, spec, cuda, seed_base, f"#long{kind}4")
    ok = one.resident_ok(s1, B) if kind == "resident" else one.hybrid_ok(s1, B)
    assert ok
    if kind == "resident":
        l1 = one.run_resident_epoch(acts, labels, s1, B)
        l2 = torch.cat([chunked.run_resident_epoch(acts[i * B:(i + CHUNK) * B], labels[i * B:(i + CHUNK) * B], s2, B)
                        for i in range(0, STEPS, CHUNK)])
    else:
        l1 = one.run_hybrid_epoch(acts, labels, s1, B)
        chunked.hybrid_chunk_steps = CHUNK               # the executor's own chunked launches
        assert chunked._hybrid_executor(s2, B).max_steps() == CHUNK
        l2 = chunked.run_hybrid_epoch(acts, labels, s2, B)
        assert one._hybrid_executor(s1, B).max_steps() >= STEPS
    l3 = _launch_per_stage_epoch(lps, s3, acts, labels, B)
    l4 = _launch_per_stage_epoch(ctl, s4, _ulp(acts), labels, B)
    torch.cuda.synchronize()
    a, b, c, d = _tail_states(one, s1), _tail_states(chunked, s2), _tail_states(lps, s3), _tail_states(ctl, s4)
    assert torch.equal(l1, l2)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert torch.isfinite(l1).all()
    _check_close(f"{kind} {STEPS} steps vs launch-per-stage", a, c, d, l1, l3, l4)
    assert (one.fwd_count, s1.t) == (chunked.fwd_count, s2.t) == (lps.fwd_count, s3.t) == (STEPS, STEPS)


def test_vanilla_epoch_long_launch(cuda, tmp_path):
    B = 16
    s1 = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    s2 = _session("vanilla", tmp_path, True, cuda, B, persist=True)
    sp = _session("vanilla", tmp_path, True, cuda, B)
    sc = _session("vanilla", tmp_path, True, cuda, B)
    with torch.no_grad():                         # the control: Bob's fc1 moved by one ulp
        sc.tail.layers[0].W.copy_(_ulp(sc.tail.layers[0].W))
    s2._va_max_steps = CHUNK
    tr = s1.alices[1].train
    reps = -(-(STEPS * B + 7) // len(tr.y))
    order = torch.cat([tr.shuffled_order(torch.Generator().manual_seed(40 + r)) for r in range(reps)])
    order = order[:STEPS * B + 7].to(cuda)        # 1,000 full batches + a short one
    for s in (s1, s2, sp, sc):
        s.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    assert s1.native_split_epochs.get("persistent") == 1 and s2.native_split_epochs.get("persistent") == 1
    a, b, c, d = _states(s1, "vanilla"), _states(s2, "vanilla"), _states(sp, "vanilla"), _states(sc, "vanilla")
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert all(torch.isfinite(v).all() for v in a.values())
    z = torch.zeros(CHUNK * B)
    _check_close(f"vanilla {STEPS + 1} steps vs per-batch", a, c, d, z, z, z)
    assert s1.tail.fwd_count == sp.tail.fwd_count == STEPS + 1
