"""Headline benchmark: whole-node samples/s of the SISA split-learning pipeline.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (N > 1; one rank per GPU)

Metric (BASELINE.json): "samples/sec (whole node) split-NN MNIST, world_size=2/3/5/9
on 1/2/4/8 MI355X".  With N GPUs the job has world_size = N + 1 roles: N Alices
(one per GPU) and Bob, whose server tail is tensor-parallel over all N GPUs.

One timed step = one full SISA round with the reference's semantics
(split_nn.py:74-95, data_entities_vanilla_sisa.py): every Alice trains her conv
front for one local epoch over her shard (all Alices concurrently, Adam), the
fronts are frozen, the activation cache is rebuilt (each Alice's shard through the
frozen front, multicast to every Bob rank), and Bob trains one server epoch over
all cached activations (Adam wd=1e-5, batch 16, one optimizer step per batch).
Every training sample therefore passes one Alice-local step and one Bob step;
value = (N * samples_per_client) / seconds per round, summed over the node.
Per-Alice work is fixed as N grows ("weak" scaling).  Data: synthetic
MNIST-shaped uint8 images (learnable class prototypes), random-init weights of
the reference architectures (model1_sisa + model2_sisa), fp32 parameters and
optimizer state, fp32 MFMA compute (higher precision than bf16; the step is
HBM-bound, so fp32 costs no time).

vs_baseline divides by the reference's own CPU number for the same pipeline at
world_size 2 (5,600 samples through the SISA local + server phases
in 10.536 s + 71.264 s = 68.46 samples/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np
import torch
import torch.distributed as dist

BASELINE_SAMPLES_PER_S = 5600.0 / (10.536 + 71.264)
# per-mode reference numbers (CPU): vanilla ws=2 train phase 5,600 / 32.126 s;
# the reference's U-shape and concat modes crash, so they have none
BASELINES = {"sisa": BASELINE_SAMPLES_PER_S, "vanilla": 5600.0 / 32.126, "ushape": None, "concat": None}
METRIC = "samples/sec (whole node) split-NN MNIST, world_size=2/3/5/9 on 1/2/4/8 MI355X"
MODELS = {
    "sisa": "model1_sisa (Alice) + model2_sisa (Bob), SISA round (split_nn.py --sisa)",
    "concat": "model1_sisa (Alices) + model2_sisa_concat(k) (Bob), SISA-concat round (--sisa --concat)",
    "vanilla": "model1_sisa (Alice) + model2_sisa (Bob), SGD-m, round-robin iteration (--vanilla)",
    "ushape": "model1 + model3 (Alice) + model2 (Bob), Adam, round-robin iteration (U-shape default)",
}


def _session_args(a, world_size, log_dir):
    return SimpleNamespace(
        world_size=world_size, client_num_in_total=world_size - 1, epochs=a.epochs, iterations=1,
        batch_size=a.batch_size, partition_alpha=0.5, datapath="", lr=1e-3, server_epochs=a.server_epochs,
        vanilla=a.mode == "vanilla", sisa=a.mode in ("sisa", "concat"), concat=a.mode == "concat", control=False,
        mode=a.mode, seed=a.seed, log_dir=log_dir,
        no_tqdm=True, true_reset=False, eval_dropout_fix=False, concat_unlearn=False, omit_label=9,
        unlearn_client_ids=[1], save_dir="", resume_dir="", kernels=a.kernels, graphs=a.graphs,
        act_dtype=a.act_dtype)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples_per_client", type=int, default=2048)
    ap.add_argument("--batch_size", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--server_epochs", type=int, default=1)
    ap.add_argument("--kernels", choices=("auto", "hip", "torch"), default="auto")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--bob_tp", type=int, default=0, help="0 = all ranks")
    ap.add_argument("--json_out", type=str, default="")
    ap.add_argument("--graphs", choices=("auto", "on", "off"), default="auto")
    ap.add_argument("--act_dtype", choices=("fp32", "bf16"), default="fp32",
                    help="SISA activation-cache storage dtype (compute stays fp32)")
    ap.add_argument("--mode", choices=("sisa", "vanilla", "ushape", "concat"), default="sisa",
                    help="sisa (headline): one SISA round; vanilla / ushape: one round-robin "
                         "iteration (every Alice one epoch of split training, weight relay); "
                         "concat: one SISA-concat round")
    ap.add_argument("--kernel_variant", action="append", default=[], metavar="SLOT=VALUE",
                    help="A/B hook: select a measured-alternative kernel form (_C.set_variant)")
    a = ap.parse_args(argv)

    from splitlearning_amd import ops
    from splitlearning_amd.data.mnist import synthetic_mnist
    from splitlearning_amd.parallel.dist import Comm, Placement, make_tp_group
    from splitlearning_amd.protocols import SESSIONS

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
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    if world > 1:
        import datetime
        kw = {"device_id": dev} if use_gpu else {}
        dist.init_process_group("nccl" if use_gpu else "gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=900), **kw)
    N = world
    ws = N + 1
    pl = Placement.make(ws, N, a.bob_tp if a.bob_tp > 0 else N)
    comm = Comm(rank, N, dev, pl, make_tp_group(pl, "nccl" if use_gpu else "gloo") if N > 1 else None)
    S = a.samples_per_client

    class BenchSession(SESSIONS[a.mode]):
        def _load_client_shard(self, cid):
            x, y = synthetic_mnist(S + 256, seed=1000 + cid)
            return ({"x": torch.from_numpy(x[:S]), "y": torch.from_numpy(y[:S])},
                    {"x": torch.from_numpy(x[S:]), "y": torch.from_numpy(y[S:])})

    log_dir = os.path.join("/tmp", f"sl_bench_logs_{os.getpid()}")
    sess = BenchSession(_session_args(a, ws, log_dir), comm, dev)
    k = ws - 1
    all_alices = range(1, k + 1)

    def step():
        if a.mode in ("vanilla", "ushape"):
            for cid in all_alices:             # split_nn.py:49-52, one iteration
                sess.train_request(cid)
            return
        sess.train_request_parallel()
        sess.freeze_alice_weights(all_alices)
        sess.reset_activation_cache()          # the fronts changed: rebuild the cut-layer cache
        sess.train_and_backward([], None)
        sess.unfreeze_alice_weights(all_alices)

    def sync():
        if use_gpu:
            torch.cuda.synchronize(dev)
        comm.barrier()

    for _ in range(a.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    samples = k * S * a.steps
    value = samples / dt
    if rank == 0:
        kern = "torch" if (not use_gpu or ops.get_backend() == "torch") else "hip"
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": N,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / BASELINES[a.mode], 2) if BASELINES[a.mode] else None,
            "dtype": "fp32", "data": "synthetic",
            "config": {"model": MODELS[a.mode], "mode": a.mode, "world_size": ws, "global_batch": a.batch_size,
                       "samples_per_client": S, "seq_len": None,
                       "parallelism": f"alices{k}_one_per_gpu+bob_tp{pl.bob_tp}",
                       "device": "MI355X" if use_gpu else "cpu", "kernels": kern,
                       "act_cache_dtype": a.act_dtype},
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    sess.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    _ = np
    return 0


if __name__ == "__main__":
    sys.exit(main())
