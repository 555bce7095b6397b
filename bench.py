"""Headline benchmark: whole-node samples/s of the reference's SISA job on MNIST-scale data.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (N > 1; one rank per GPU)

Metric (BASELINE.json): "samples/sec (whole node) split-NN MNIST, world_size=2/3/5/9 on
1/2/4/8 MI355X".  Config (BASELINE.json configs[3]): `split_nn.py --sisa
--server_epochs=5`, world_size = N + 1 on N GPUs: N Alices (one per GPU) and Bob, whose
server tail is tensor-parallel over all N GPUs.

Data: the reference's data volume through the reference's data path — 70,000 synthetic
MNIST-shaped uint8 images (no network for fetch_openml), Dirichlet(alpha=0.5) non-IID
partition over the N Alices and the per-client 80/20 train/test split
(`data.mnist.partition_and_split`, the same code `split_nn.py` uses), random-init weights
of the reference architectures (model1_sisa + model2_sisa), fp32 parameters, optimizer
state and compute.  The whole dataset is fixed as N grows ("strong" scaling).

One timed step = one run of the reference's whole Bob schedule for the mode
(`protocols/schedule.py` = split_nn.py:74-117 for SISA): every Alice's local epoch (all
concurrently), freeze, the activation dump into Bob's cache, `--server_epochs` Bob epochs
over all clients' cached activations, the breakdown evaluation, Alice_1's unlearning
(label 9 removed, local retrain), Bob's retraining (`--server_epochs` epochs, reusing the
other clients' cached activations) and the final evaluation.  Nothing is skipped: the
eval and unlearn phases are inside the timed region.

value = training samples processed per second: every sample counted once per training
epoch it passes through (Alice-local or Bob-server), eval samples not counted (their time
is).  The reference publishes no number; BASELINE.md measured its phase rates on CPU
(SISA ws=2: Alice local 531.5, Bob server 78.6, Bob retrain 90.5 samples/s).
vs_baseline divides by those rates composed over THIS schedule's sample counts
(reference eval time counted as zero, in its favour); config.baseline_samples_per_s
records the composed number.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

METRIC = "samples/sec (whole node) split-NN MNIST, world_size=2/3/5/9 on 1/2/4/8 MI355X"
# reference CPU phase rates, samples/s, by schedule phase kind
REF_RATES = {
    "sisa": {"local": 531.5, "server": 78.6, "retrain": 90.5},
    "control": {"local": 531.5, "server": 78.6, "retrain": 90.5},
    "vanilla": {"train": 5600.0 / 32.126},
    "ushape": None,          # the reference's U-shape crashes (Q1)
    "concat": None,          # the reference's concat crashes (Q3)
}
MODELS = {
    "sisa": "model1_sisa (Alice) + model2_sisa (Bob), split_nn.py --sisa",
    "control": "model1_sisa (Alice) + model2_sisa (Bob), split_nn.py --control",
    "concat": "model1_sisa (Alices) + model2_sisa_concat(k) (Bob), split_nn.py --sisa --concat",
    "vanilla": "model1_sisa (Alice) + model2_sisa (Bob), SGD-m, split_nn.py --vanilla",
    "ushape": "model1 + model3 (Alice) + model2 (Bob), Adam, split_nn.py (U-shape default)",
}
MODE_FLAGS = {"sisa": ["--sisa"], "control": ["--control"], "concat": ["--sisa", "--concat"],
              "vanilla": ["--vanilla"], "ushape": []}


def _phase_kind(mode: str, name: str):
    """Map a schedule phase to the reference rate that prices it (None = not a training phase)."""
    if mode in ("sisa", "control", "concat"):
        if name.startswith("server_retraining"):
            return "retrain"
        if name.startswith("server_training"):
            return "server"
        if name.startswith(("local_training", "unlearn_local", "control_local")):
            return "local"
        return None
    if name.startswith(("train_request", "unlearn_request")):
        return "train"
    return None


def _ipc_status():
    """The peer-mapped TP all-reduce's set-up outcome on this process (parallel/rccl.py)."""
    from splitlearning_amd.parallel.rccl import IPC_STATUS
    return dict(IPC_STATUS) if IPC_STATUS else None


def _channel_kind(sess):
    ch = getattr(sess, "split_channel", None)
    if ch is None:
        return None
    return "ipc" if hasattr(ch, "host_error") else "rccl"


def _gathered_split(sess):
    """Native split epochs by kind, summed over the ranks (gathered before rank 0 reports)."""
    tot = {}
    for d in getattr(sess, "_split_counts_all", None) or []:
        for k, v in (d or {}).items():
            tot[k] = tot.get(k, 0) + v
    return tot


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=tuple(MODE_FLAGS), default="sisa")
    ap.add_argument("--schedule", choices=("full", "round"), default="full",
                    help="full: the mode's whole split_nn.py schedule; round (SISA modes): local "
                         "training + the server epochs only")
    ap.add_argument("--world_size", type=int, default=0, help="0 = gpus + 1 (BASELINE configs)")
    ap.add_argument("--server_epochs", type=int, default=5, help="BASELINE config 4: --server_epochs=5")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--iterations", type=int, default=1, help="round-robin rounds (vanilla / U-shape)")
    ap.add_argument("--batch_size", type=int, default=16)
    ap.add_argument("--num_samples", type=int, default=70000, help="MNIST size (train + test)")
    ap.add_argument("--partition_alpha", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--kernels", choices=("auto", "hip", "torch"), default="auto")
    ap.add_argument("--bob_tp", type=int, default=0,
                    help="0 = the policy (parallel/dist.py choose_bob_tp: all GPUs for the SISA modes)")
    ap.add_argument("--graphs", choices=("auto", "on", "off"), default="auto")
    ap.add_argument("--hybrid", choices=("auto", "off"), default="auto",
                    help="SISA server epochs of a wide Bob shard (TP <= 4) on the hybrid persistent "
                         "executor (csrc/hybrid.hip: fc2 / fc3 on-chip, fc1 streamed in one launch)")
    ap.add_argument("--resident", choices=("auto", "off"), default="auto",
                    help="SISA server epochs of a narrow Bob shard (TP >= 7) on the register-resident "
                         "persistent executor (csrc/resident.hip) after its cross-rank self-test")
    ap.add_argument("--split_persist", choices=("auto", "off"), default="auto",
                    help="vanilla: co-located epochs as one persistent launch (csrc/vanilla.hip)")
    ap.add_argument("--tp_allreduce", choices=("auto", "rccl"), default="auto",
                    help="Bob's TP all-reduce: peer-mapped one-kernel path when it passes set-up (auto) or RCCL")
    ap.add_argument("--act_dtype", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32", help="compute dtype")
    ap.add_argument("--concat_unlearn", action="store_true", default=True,
                    help="concat: add the unlearning retrain (BASELINE config 5)")
    ap.add_argument("--python_epoch", action="store_true",
                    help="A/B: epochs as Python loops instead of the native executors")
    ap.add_argument("--json_out", type=str, default="")
    ap.add_argument("--ranks_share_gpu", action="store_true",
                    help="rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, gloo "
                         "control + host-staged data plane, Bob's TP all-reduce peer-mapped (RCCL "
                         "refuses two ranks on one device).  Not a scaling measurement.")
    ap.add_argument("--kernel_variant", action="append", default=[], metavar="SLOT=VALUE",
                    help="A/B hook: select a measured-alternative kernel form (_C.set_variant)")
    a = ap.parse_args(argv)

    from splitlearning_amd import ops
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import make_client_shards, synthetic_mnist
    from splitlearning_amd.parallel.dist import Comm, Placement, choose_bob_tp, make_tp_group
    from splitlearning_amd.protocols import SESSIONS
    from splitlearning_amd.protocols.schedule import build_steps

    if a.kernels == "torch":
        ops.set_backend("torch")
    for kv in a.kernel_variant:
        from splitlearning_amd.ops import hip_ops
        slot, val = (int(v) for v in kv.split("="))
        hip_ops.C().set_variant(slot, val)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1 and world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    use_gpu = torch.cuda.device_count() > 0
    share = a.ranks_share_gpu and use_gpu and world > 1
    dev = torch.device("cuda", 0 if share else local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    backend = "nccl" if use_gpu and not share else "gloo"
    if world > 1:
        import datetime
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=900), **kw)
    N = world
    ws = a.world_size if a.world_size > 0 else N + 1
    log_dir = os.path.join("/tmp", f"sl_bench_logs_{os.getpid()}")
    argv_s = MODE_FLAGS[a.mode] + [
        "--world_size", str(ws), "--epochs", str(a.epochs), "--iterations", str(a.iterations),
        "--batch_size", str(a.batch_size), "--partition_alpha", str(a.partition_alpha),
        "--server_epochs", str(a.server_epochs), "--seed", str(a.seed), "--num_samples", str(a.num_samples),
        "--kernels", a.kernels, "--graphs", a.graphs, "--act_dtype", a.act_dtype, "--dtype", a.dtype, "--no_tqdm",
        "--tp_allreduce", a.tp_allreduce, "--resident", a.resident, "--hybrid", a.hybrid,
        "--split_persist", a.split_persist, "--log_dir", log_dir, "--watchdog", "off"]
    if a.mode == "concat" and a.concat_unlearn:
        argv_s.append("--concat_unlearn")
    if a.python_epoch:
        argv_s.append("--python_epoch")
    sargs = parse_args(argv_s)
    pl = Placement.make(ws, N, a.bob_tp if a.bob_tp > 0 else (choose_bob_tp(sargs.mode, N) if use_gpu else N))
    comm = Comm(rank, N, dev, pl, make_tp_group(pl, backend) if N > 1 else None)
    comm.host_staging = share
    k = ws - 1

    # the reference's data volume and data path: one MNIST-sized set, Dirichlet-partitioned
    x, y = synthetic_mnist(a.num_samples, seed=a.seed)
    shards = make_client_shards(x, y, k, a.partition_alpha, seed=a.seed)
    del x, y

    class BenchSession(SESSIONS[sargs.mode]):
        def _load_client_shard(self, cid):
            xtr, ytr, xte, yte = shards[cid]
            return ({"x": torch.from_numpy(xtr), "y": torch.from_numpy(ytr)},
                    {"x": torch.from_numpy(xte), "y": torch.from_numpy(yte)})

    sess = BenchSession(sargs, comm, dev)
    sess.quiet = True                  # stdout carries the one JSON line only
    all_alices = list(range(1, k + 1))
    steps = build_steps(sess, sargs)
    if a.schedule == "round":
        if sargs.mode not in ("sisa", "concat", "control"):
            raise SystemExit("--schedule round is a SISA-mode schedule")
        steps = [(n, f) for n, f in steps if n in ("local_training", "server_training")]

    calib = None
    if N > 1:
        # measured link costs on this job's ranks and transport (not timed): the split modes'
        # per-batch act / cut-gradient message and Bob's TP all-reduce (parallel/calibrate.py)
        from splitlearning_amd.parallel.calibrate import measure
        tail = getattr(sess, "tail", None)
        calib = measure(comm, dev, a.batch_size, allreduce=tail.allreduce if tail is not None else None,
                        tp_ranks=pl.bob_ranks if pl.bob_tp > 1 else ())
        if calib and calib.get("msg_us") is not None:
            calib["bob_tp_policy"] = {m: choose_bob_tp(m, N, calib["msg_us"]) for m in ("vanilla", "ushape")}

    def step():
        # a fresh repetition of the schedule: fronts trainable, Bob's cut-layer cache empty
        # (the fronts change every repetition); weights and optimizer state carry on
        sess.reset_activation_cache()
        sess.unfreeze_alice_weights(all_alices)
        for _, fn in steps:
            fn()

    def sync():
        if use_gpu:
            torch.cuda.synchronize(dev)
        comm.barrier()

    for _ in range(a.warmup):
        step()
    sync()
    rec0 = len(sess.timer.records)
    b0 = comm.bytes_sent
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    recs = sess.timer.records[rec0:]
    samples = 0
    phase_s, phase_n = {}, {}
    for r in recs:
        key = r["phase"].split("[")[0]
        phase_s[key] = phase_s.get(key, 0.0) + r["seconds"] / a.steps
        if _phase_kind(sargs.mode, r["phase"]) is not None:
            samples += r["samples"]
            phase_n[key] = phase_n.get(key, 0) + r["samples"] // a.steps
    value = samples / dt
    rates = REF_RATES.get(sargs.mode)
    base = None
    if rates is not None and samples:
        ref_t = sum(r["samples"] / rates[_phase_kind(sargs.mode, r["phase"])] for r in recs
                    if _phase_kind(sargs.mode, r["phase"]) is not None)
        base = samples / ref_t
    # after the clock: is what the adopted server executor computed right?  (every rank joins;
    # the persistent executor replays a slice against launch-per-stage from one snapshot, the
    # replicated fc3 is compared across Bob ranks; the job's state is restored afterwards)
    from splitlearning_amd.engine.resident import validate
    val = validate(sess)
    sent = comm.gather_obj((comm.bytes_sent - b0) // max(1, a.steps), 0)
    sess._split_counts_all = comm.gather_obj(dict(getattr(sess, "native_split_epochs", {})), 0)
    if rank == 0:
        kern = "torch" if (not use_gpu or ops.get_backend() == "torch") else "hip"
        tpc = getattr(sess, "tp_native_comm", None)
        flags = " ".join(MODE_FLAGS[a.mode] + [f"--server_epochs={a.server_epochs}", f"--world_size={ws}",
                                                f"--batch_size={a.batch_size}", f"--epochs={a.epochs}"])
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": N,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3),
            "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(value / base, 2) if base else None,
            "dtype": a.dtype, "data": "synthetic",
            "config": {
                "model": MODELS[sargs.mode], "mode": sargs.mode, "flags": flags, "world_size": ws,
                "global_batch": a.batch_size, "seq_len": None, "schedule": a.schedule,
                "num_samples": a.num_samples, "partition": f"dirichlet(alpha={a.partition_alpha}) + 80/20 split",
                "train_samples_per_client": {c: int(len(shards[c][1])) for c in all_alices},
                "parallelism": f"alices{k}_on_{N}gpus+bob_tp{pl.bob_tp}",
                "device": "MI355X" if use_gpu else "cpu", "ranks_share_gpu": share,
                "kernels": kern, "act_cache_dtype": a.act_dtype,
                "train_samples_per_step": samples // a.steps,
                "phase_seconds": {p: round(v, 4) for p, v in phase_s.items()},
                "phase_train_samples": phase_n,
                "baseline_samples_per_s": round(base, 2) if base else None,
                "baseline_basis": ("reference CPU phase rates from BASELINE.md composed over this schedule's "
                                   "sample counts" if base else None),
                "dist_world": N, "rccl_nranks": int(tpc.size) if tpc is not None else (1 if use_gpu and N == 1 else 0),
                "tp_allreduce": ("ipc" if getattr(sess, "tp_ipc", None) is not None else
                                 "rccl" if tpc is not None else "torch.distributed" if N > 1 else "none"),
                "bytes_sent_per_rank_per_step": sent,
                "tp_ipc_setup": _ipc_status(),
                # Bob's server-epoch executor: the register-resident persistent launch (a shard
                # narrow enough to keep on-chip, its self-test passed) or the launch-per-stage one
                "server_executor": getattr(sess, "server_executor", "launch_per_stage")
                if sargs.mode in ("sisa", "control") else None,
                # why: adopted, or the fit / self-test outcome that kept launch-per-stage
                "server_executor_reason": (getattr(sess, "resident_status", None) or {}).get("reason"),
                # a persistent epoch that failed mid-launch: rolled back, the job continued on
                # launch-per-stage from that client epoch on ({from, epoch, reason}; None: none)
                "server_executor_fallback": (getattr(sess, "resident_status", None) or {}).get("fallback"),
                # the post-run self-check (engine/resident.validate): None = nothing to check
                # for this mode; details: replayed steps, loss / fc3 gaps, fc3 replicas equal
                "validated": val.get("validated"),
                "validation": val,
                "calib": calib,
                # vanilla / U-shape: the native split epochs this rank ran (co-located, or its
                # side of a remote Alice's) and the per-batch link of the remote ones
                "split_epochs": _gathered_split(sess) if sargs.mode in ("vanilla", "ushape") else None,
                "split_persist_fallback": (getattr(sess, "split_persist_fallback", None)
                                           or getattr(sess, "split_persist_reason", None)),
                "split_channel": _channel_kind(sess) if sargs.mode in ("vanilla", "ushape") else None,
            },
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    sess.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
