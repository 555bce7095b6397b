"""Multi-process protocol tests on CPU (gloo): the distributed paths the 8-GPU node runs,
exercised here with 2-3 processes.

* tensor-parallel Bob (TP=2) equals the single-process Bob step for step;
* every mode runs end-to-end through the real launcher with one process per role
  (reference topology) and with fewer processes than roles (Alices co-located,
  Bob tensor-parallel) — the MI355X placement;
* log vocabulary and metrics are produced.
"""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from splitlearning_amd.runtime.launcher import main as launch_main


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, out_dir, steps):
    import torch.distributed as dist
    from splitlearning_amd.config import OptimCfg
    from splitlearning_amd.engine import OptSlot, TailEngine
    from splitlearning_amd.models import ServerTailSisa, sisa_server_spec
    from splitlearning_amd.ops import torch_ops as K
    from splitlearning_amd.parallel.dist import Comm, Placement, make_tp_group
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pl = Placement.make(world + 1, world, world)
    comm = Comm(rank, world, torch.device("cpu"), pl, make_tp_group(pl, "gloo"))
    torch.manual_seed(0)
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), torch.device("cpu"), rank, world,
                      allreduce=comm.tp_allreduce, seed_base=3)
    slot = OptSlot(OptimCfg("adam", 1e-3, weight_decay=1e-5))
    g = torch.Generator().manual_seed(1)
    outs = []
    for _ in range(steps):
        x = torch.rand(16, 5408, generator=g) * 20
        y = torch.randint(0, 10, (16,), generator=g)
        o = tail.forward(x, train=True)
        _, d = K.softmax_ce(o, y, 1 / 16)
        dx = tail.backward_dgrad(d, need_dx=True)
        dx = comm.reduce_to(dx, 0, pl.bob_ranks, dx.shape, dx.dtype)
        tail.backward_step(slot)
        if rank == 0:
            outs.append((o.clone(), dx.clone()))
    sd = tail.full_state_dict(comm.tp_allgather)
    if rank == 0:
        torch.save({"sd": sd, "outs": outs}, os.path.join(out_dir, f"tp{world}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_tensor_parallel_bob_matches_single_process(tmp_path):
    steps = 3
    mp.spawn(_tp_worker, args=(2, _free_port(), str(tmp_path), steps), nprocs=2, join=True)
    mp.spawn(_tp_worker, args=(1, _free_port(), str(tmp_path), steps), nprocs=1, join=True)
    a = torch.load(tmp_path / "tp2.pt", weights_only=True)
    b = torch.load(tmp_path / "tp1.pt", weights_only=True)
    for (o2, dx2), (o1, dx1) in zip(a["outs"], b["outs"]):
        torch.testing.assert_close(o2, o1, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(dx2, dx1, rtol=1e-4, atol=1e-5)
    for k in b["sd"]:
        d = (a["sd"][k] - b["sd"][k]).abs()
        assert a["sd"][k].shape == b["sd"][k].shape, k
        assert d.max().item() < 7e-3 and (d > 1e-5).float().mean().item() < 1e-4, k


def _run(tmp_path, mode_flags, world_size, nprocs, bob_tp=1, extra=(), seed=3):
    logs = tmp_path / "logs"
    seed_args = [] if seed is None else ["--seed", str(seed)]
    argv = list(mode_flags) + ["--world_size", str(world_size), "--nprocs", str(nprocs), "--bob_tp", str(bob_tp),
                               "--iterations", "1", "--server_epochs", "1", "--num_samples", "700"] + seed_args + [
                               "--no_tqdm", "--device", "cpu", "--datapath", str(tmp_path / "data"),
                               "--log_dir", str(logs), "--master_port", str(_free_port())] + list(extra)
    launch_main(argv)
    with open(logs / "metrics.json") as f:
        m = json.load(f)
    bob = (logs / "bob.log").read_text()
    return m, bob, logs


@pytest.mark.slow
@pytest.mark.parametrize("flags,ws,np_,tp", [
    (["--vanilla"], 3, 3, 1),          # reference topology: 1 process per role
    (["--vanilla"], 3, 2, 2),          # MI355X placement: Alices co-located, Bob TP=2
    ([], 3, 2, 2),                     # U-shape
    (["--sisa"], 3, 2, 2),
    (["--sisa", "--act_dtype", "bf16"], 3, 3, 2),   # bf16 activation cache over p2p
    (["--vanilla", "--act_dtype", "bf16"], 3, 3, 2),  # bf16 cut activations on the wire
    (["--act_dtype", "bf16"], 3, 2, 2),              # U-shape, bf16 wire
    (["--control"], 3, 3, 1),
    (["--sisa", "--concat", "--concat_unlearn"], 3, 2, 2),
])
def test_modes_end_to_end(tmp_path, flags, ws, np_, tp):
    m, bob, logs = _run(tmp_path, flags, ws, np_, tp)
    assert "Bob Started Getting Tipsy" in bob
    assert "Accuracy over all data" in bob
    assert m["nprocs"] == np_ and m["bob_tp"] == tp
    for cid in range(1, ws):
        alog = (logs / f"alice{cid}.log").read_text()
        assert "Alice is going insane!" in alog and "Local Data Statistics:" in alog
    if "--vanilla" in flags:
        assert "Train Request for Alice-1" in bob and "Unlearn Request for Alice-1" in bob
        assert "receiving weights from Alice-1" in (logs / "alice2.log").read_text()
    if "--sisa" in flags and "--concat" not in flags:
        for line in ["Train all Alices in parallel", "Server training starts. Freezing weights for Alices-1.",
                     "Global Training", "Global training completed.", "Unfreezing weights for Alices-1.",
                     "Unlearn Request for Alice-1 upon the label-9"]:
            assert line in bob, line
        assert "Unlearning label: 9, and reset the model" in (logs / "alice1.log").read_text()
    if "--control" in flags:
        assert "Filtered dataset:" in (logs / "alice1.log").read_text()


@pytest.mark.slow
def test_checkpoint_roundtrip(tmp_path):
    ck = tmp_path / "ck"
    _run(tmp_path, ["--vanilla"], 3, 2, 2, extra=["--save_dir", str(ck)])
    bob = torch.load(ck / "bob.pt", weights_only=True)
    assert tuple(bob["fc1.weight"].shape) == (5000, 5408) and tuple(bob["fc2.weight"].shape) == (1000, 5000)
    a1 = torch.load(ck / "alice1.pt", weights_only=True)
    assert set(a1) == {"conv_layers.0.weight", "conv_layers.0.bias"}
    # resume into a fresh run: loads without error and trains on
    _run(tmp_path, ["--vanilla"], 3, 2, 2, extra=["--resume_dir", str(ck)])


@pytest.mark.slow
@pytest.mark.parametrize("nranks", [2, 4])
def test_bench_multi_rank_gloo(tmp_path, nranks):
    """bench.py under torch.distributed.run with 2 and 4 CPU ranks (gloo): one JSON line
    from rank 0 with the driver's contract fields and the multi-rank evidence fields (the
    GPU path is the same code over RCCL)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "b.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(nranks), "--steps", "1", "--warmup", "1", "--num_samples", str(300 * nranks),
           "--server_epochs", "1", "--json_out", str(out)]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    # gloo itself prints "[Gloo] Rank r is connected ..." lines (other processes, possibly
    # interleaved); ours is the one JSON line
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec == json.loads(out.read_text())
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    c = rec["config"]
    assert rec["n_gpus"] == nranks and rec["value"] > 0 and c["world_size"] == nranks + 1
    assert c["dist_world"] == nranks and len(c["bytes_sent_per_rank_per_step"]) == nranks
    assert c["parallelism"].endswith(f"bob_tp{nranks}")
    # the whole schedule ran: training, eval and unlearning phases are all timed
    for p in ("local_training", "server_training", "eval_breakdown", "unlearn_local", "server_retraining"):
        assert p in c["phase_seconds"], p
    # the SISA dump crossed ranks (Alices on ranks 1.. multicast to every Bob TP rank)
    assert sum(c["bytes_sent_per_rank_per_step"]) > 0
    # self-calibration: the per-batch message cost to every peer and the TP all-reduce cost
    cal = c["calib"]
    assert cal["msg_us"] > 0 and sorted(cal["per_peer_us"]) == [str(r) for r in range(1, nranks)]
    assert cal["tp_allreduce_us"] > 0 and set(cal["bob_tp_policy"]) == {"vanilla", "ushape"}


@pytest.mark.slow
@pytest.mark.parametrize("flags,np_,tp,crash_at", [
    (["--sisa"], 2, 2, "1:unlearn_local:crash"),          # TP=2 Bob shards, co-located Alices
    (["--vanilla"], 3, 1, "2:unlearn_request[1]:crash"),  # one process per role
])
def test_crash_and_resume_matches_uninterrupted(tmp_path, flags, np_, tp, crash_at):
    """--ckpt_dir snapshots after every schedule step; a job killed mid-schedule (fault
    injection: a rank crashes at a phase beacon) and restarted with --resume finishes with
    weights bitwise equal to an uninterrupted run and the same final evaluation."""
    ref, run = tmp_path / "ref", tmp_path / "run"
    ref.mkdir()
    run.mkdir()
    m_ref, _, _ = _run(ref, flags, 3, np_, tp, extra=["--ckpt_dir", str(ref / "ck"), "--save_dir", str(ref / "out")])
    with pytest.raises(mp.ProcessExitedException):
        _run(run, flags, 3, np_, tp, extra=["--ckpt_dir", str(run / "ck"), "--fault_inject", crash_at])
    done = int((run / "ck" / "latest").read_text())
    assert done >= 1
    m_res, bob, _ = _run(run, flags, 3, np_, tp,
                         extra=["--ckpt_dir", str(run / "ck"), "--resume", "--save_dir", str(run / "out")])
    assert f"[resume] {done} of" in bob
    assert m_res["last_eval"] == m_ref["last_eval"]
    for f in ["bob.pt", "alice1.pt", "alice2.pt"]:
        a = torch.load(ref / "out" / f, weights_only=True)
        b = torch.load(run / "out" / f, weights_only=True)
        flat_a = a if "model1" not in a else {**a["model1"], **a["model3"]}
        flat_b = b if "model1" not in b else {**b["model1"], **b["model3"]}
        assert flat_a.keys() == flat_b.keys()
        for k in flat_a:
            assert torch.equal(flat_a[k], flat_b[k]), (f, k)
    # snapshots are pruned to --ckpt_keep and loadable without unpickling code
    steps = sorted(p.name for p in (run / "ck").iterdir() if p.name.startswith("step"))
    assert len(steps) <= 2
    torch.load(run / "ck" / steps[-1] / "rank0.pt", weights_only=True)


@pytest.mark.slow
def test_resume_without_seed_flag(tmp_path):
    """A checkpointed job launched with the default flags (no --seed) records the seed it
    drew in <ckpt_dir>/job.json; --resume reuses it, so the resumed job finishes bitwise
    equal to an uninterrupted run under that seed (SISA, TP=2 Bob, co-located Alices)."""
    ref, run = tmp_path / "ref", tmp_path / "run"
    ref.mkdir()
    run.mkdir()
    flags, crash_at = ["--sisa"], "1:unlearn_local:crash"
    with pytest.raises(mp.ProcessExitedException):
        _run(run, flags, 3, 2, 2, extra=["--ckpt_dir", str(run / "ck"), "--fault_inject", crash_at], seed=None)
    seed = json.loads((run / "ck" / "job.json").read_text())["seed"]
    m_ref, _, _ = _run(ref, flags, 3, 2, 2, extra=["--save_dir", str(ref / "out")], seed=seed)
    m_res, bob, _ = _run(run, flags, 3, 2, 2, seed=None,
                         extra=["--ckpt_dir", str(run / "ck"), "--resume", "--save_dir", str(run / "out")])
    assert "[resume]" in bob
    assert m_res["last_eval"] == m_ref["last_eval"]
    for f in ["bob.pt", "alice1.pt", "alice2.pt"]:
        a = torch.load(ref / "out" / f, weights_only=True)
        b = torch.load(run / "out" / f, weights_only=True)
        for k in a:
            assert torch.equal(a[k], b[k]), (f, k)


@pytest.mark.slow
@pytest.mark.parametrize("tp", [1, 2])
def test_vanilla_per_batch_message_sequence(tmp_path, tp):
    """The split-learning data plane, pinned: one packed [activation | labels] message per
    batch from the training Alice's host to every Bob rank that is not on it, and one cut-
    gradient message per batch back from each such Bob rank (the reference needs ~4 RPC round
    trips per batch); one weight-relay message per hand-off.  Reference topology
    (one process per role, Bob on rank 0) with a TP = 1 Bob, and Bob tensor-parallel over
    ranks 0-1 (TP = 2)."""
    B = 16
    m, bob, logs = _run(tmp_path, ["--vanilla"], 3, 3, tp, extra=["--msg_log"])
    msgs = []
    for r in range(3):
        msgs += [tuple(x) for x in json.loads((logs / f"messages_rank{r}.json").read_text())]
    import math
    from splitlearning_amd.data.mnist import load_shard
    data = tmp_path / "data"
    n_tr = {c: int(load_shard(str(data), c)[0]["y"].numel()) for c in (1, 2)}
    y1 = load_shard(str(data), 1)[0]["y"]
    n_unl = int((y1 != 9).sum())
    bob_ranks = list(range(tp))

    from splitlearning_amd.protocols.base import Session
    # [M x 5408 activation | M int64 labels], padded to 16-byte units (Session.pack)
    pack_bytes = {4 * Session.packed_len(M, torch.float32) for M in range(1, B + 1)}

    def packs(src, dst):
        return [x for x in msgs if x[0] == "multicast" and x[1] == src and x[2] == dst and x[3] in pack_bytes]

    def grads(src, dst):
        return [x for x in msgs if x[0] == "reduce_to" and x[1] == src and x[2] == dst]
    # Alice_c lives on rank c; batches of train_request(c), plus Alice_1's unlearn epoch
    for c in (1, 2):
        nb = math.ceil(n_tr[c] / B) + (math.ceil(n_unl / B) if c == 1 else 0)
        for b in bob_ranks:
            if b == c:
                continue
            assert len(packs(c, b)) == nb, (c, b, len(packs(c, b)), nb)
            assert len(grads(b, c)) == nb, (c, b, len(grads(b, c)), nb)
            assert all(x[3] <= 4 * B * 5408 for x in grads(b, c))
    # the round-robin hand-off Alice_1 -> Alice_2: one flat 320-float buffer
    relay = [x for x in msgs if x[0] == "send_recv" and x[1] == 1 and x[2] == 2 and x[3] == 4 * 320]
    assert len(relay) == 1
    # nothing else goes Bob -> Alice per batch
    assert not [x for x in msgs if x[0] == "multicast" and x[1] in bob_ranks and x[2] in (1, 2)
                and x[3] >= 4 * B * 5408 and x[1] != x[2] and x[1] not in (1, 2)]


@pytest.mark.slow
@pytest.mark.parametrize("flags,ws,np_,tp", [
    (["--vanilla"], 3, 3, 2),                 # per-batch multicast + cut-gradient reduce + relay
    (["--sisa"], 3, 2, 2),                    # the batched dump exchange, eval traffic
    ([], 3, 3, 1),                            # U-shape: four messages per batch
    (["--sisa", "--concat", "--concat_unlearn"], 3, 3, 2),
])
def test_native_data_plane_protocol_matches_torch_p2p(tmp_path, flags, ws, np_, tp):
    """The GPU data plane (Comm.native: grouped RCCL p2p on the compute stream) with RCCL's
    ordering semantics, run over gloo (GlooP2PShim): the protocol completes (no stream-order
    deadlock) and the job is bitwise the torch.distributed p2p run."""
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    m_ref, _, _ = _run(a, flags, ws, np_, tp, extra=["--save_dir", str(a / "out")])
    m_nat, _, _ = _run(b, flags, ws, np_, tp, extra=["--native_p2p_shim", "--save_dir", str(b / "out")])
    assert m_nat["last_eval"] == m_ref["last_eval"]
    for f in sorted(p.name for p in (a / "out").iterdir()):
        x = torch.load(a / "out" / f, weights_only=True)
        y = torch.load(b / "out" / f, weights_only=True)
        fx = x if "model1" not in x else {**x["model1"], **x["model3"]}
        fy = y if "model1" not in y else {**y["model1"], **y["model3"]}
        for k in fx:
            assert torch.equal(fx[k], fy[k]), (f, k)


def _ipc_fallback_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splitlearning_amd.parallel.rccl import make_ipc_allreduce
    # no GPU here: the region allocation fails on every member, so all ranks (members or
    # not) must come back with None together rather than hang in the handle exchange
    got = make_ipc_allreduce([0, 1], rank)
    with open(os.path.join(out_dir, f"ipc{rank}.txt"), "w") as f:
        f.write("none" if got is None else "up")
    dist.barrier()
    dist.destroy_process_group()


def test_ipc_allreduce_setup_falls_back_together(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_ipc_fallback_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    assert [open(tmp_path / f"ipc{r}.txt").read() for r in range(3)] == ["none"] * 3
