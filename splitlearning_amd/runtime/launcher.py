"""Process launcher: argument resolution, data generation, process spawn, per-rank entry.

Reference: `split_nn.py:148-186` (argparse, validation, `load_mnist_image`, then
`mp.spawn(example, nprocs=world_size)`) and `example()` (`:34-146`).

MI355X mapping:
* GPU: one process per visible GPU (`--nprocs` default = #GPUs), each pinned to
  its device; roles are placed on processes (`parallel.dist.Placement`), so
  world_size = #GPUs + 1 puts Bob's TP shard and one Alice on every GPU;
* CPU: one process per role (`nprocs = world_size`), gloo, like the reference;
* already running under `torchrun` (RANK/WORLD_SIZE in the environment): no
  spawn, this process is its rank.
The parent never touches the GPU (device count only), so spawned children own it.
"""
from __future__ import annotations

import json
import os
import resource
import sys

import torch

from ..config import parse_args


def raise_fd_limit():
    """Reference split_nn.py:7-10 (needed there by TensorPipe's shm fds; harmless here)."""
    try:
        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
    except (ValueError, OSError):
        pass


def resolve(args):
    ngpu = torch.cuda.device_count() if args.device in ("auto", "cuda") else 0
    if args.device == "cuda" and ngpu == 0:
        raise RuntimeError("--device cuda but no GPU is visible")
    use_gpu = ngpu > 0
    args.use_gpu = use_gpu
    if args.nprocs <= 0:
        args.nprocs = min(ngpu, args.world_size) if use_gpu else args.world_size
    if use_gpu and args.nprocs > ngpu:
        raise RuntimeError(f"{args.nprocs} processes but only {ngpu} GPUs (one process per GPU)")
    if args.backend == "auto":
        args.backend = "nccl" if use_gpu else "gloo"
    if args.bob_tp <= 0:
        from ..parallel.dist import choose_bob_tp
        args.bob_tp_auto = True
        args.bob_tp = choose_bob_tp(args.mode, args.nprocs) if use_gpu else 1
    if args.kernels == "torch":
        from .. import ops
        ops.set_backend("torch")
    return args


def resolve_job_seed(args):
    """One agreed seed for a checkpointed job (`--ckpt_dir`).  The reference is unseeded
    (Q11) and so is a plain run here, but a snapshot only resumes under the seed that
    drew its data partition, dropout hashes and initial weights: the first run records
    the seed it used in `<ckpt_dir>/job.json` and `--resume` reads it back, so a job
    launched with the default flags (no `--seed`) can be resumed."""
    ckpt = getattr(args, "ckpt_dir", "")
    if not ckpt:
        return args
    path = os.path.join(ckpt, "job.json")
    rec = None
    if getattr(args, "resume", False) and os.path.exists(path):
        with open(path) as f:
            rec = json.load(f)
    if rec is not None:
        if args.seed is not None and int(args.seed) != int(rec["seed"]):
            raise ValueError(f"--seed {args.seed} does not match the checkpointed job's seed {rec['seed']}")
        args.seed = int(rec["seed"])
        return args
    if args.seed is None:
        import random
        args.seed = random.SystemRandom().randrange(1 << 31)
    os.makedirs(ckpt, exist_ok=True)
    with open(path + ".tmp", "w") as f:
        json.dump({"seed": int(args.seed), "mode": args.mode, "world_size": int(args.world_size)}, f)
    os.replace(path + ".tmp", path)
    return args


def worker(rank: int, nprocs: int, args, result_q=None):
    from .. import ops
    from ..parallel.dist import Comm, Placement, init_process, make_tp_group
    from ..protocols import make_session, run_schedule

    if args.kernels == "torch":
        ops.set_backend("torch")
    if args.use_gpu:
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // nprocs))
    pl = Placement.make(args.world_size, nprocs, args.bob_tp)
    tp_group = None
    if nprocs > 1:
        init_process(rank, nprocs, args.backend, args.master_addr, args.master_port, args.timeout_s, dev)
        tp_group = make_tp_group(pl, args.backend)
    if nprocs > 1 and getattr(args, "calibrate", False) and getattr(args, "bob_tp_auto", False) and args.use_gpu:
        # measured link cost -> Bob's TP degree (every rank gets rank 0's measurement, so the
        # placement agrees); the group for the policy's first guess is rebuilt
        from ..parallel.calibrate import measure
        from ..parallel.dist import choose_bob_tp
        cal = measure(Comm(rank, nprocs, dev, pl, None), dev, args.batch_size)
        args.calib = cal
        if cal.get("msg_us") is not None:
            tp = choose_bob_tp(args.mode, nprocs, cal["msg_us"])
            if tp != pl.bob_tp:
                args.bob_tp = tp
                pl = Placement.make(args.world_size, nprocs, tp)
                tp_group = make_tp_group(pl, args.backend)
    comm = Comm(rank, nprocs, dev, pl, tp_group)
    if getattr(args, "msg_log", False):
        comm.msg_log = []
    if getattr(args, "native_p2p_shim", False) and nprocs > 1:
        from ..parallel.dist import GlooP2PShim
        comm.native = GlooP2PShim()
    if getattr(args, "prep_in_worker", False) and getattr(args, "ckpt_dir", ""):
        # torchrun: every rank ran main(); rank 0's view of job.json is the agreed seed
        if rank == 0:
            resolve_job_seed(args)
        args.seed = comm.broadcast_obj(args.seed, 0)
    from .watchdog import make_watchdog
    wd = make_watchdog(args, comm)
    if wd is not None:
        comm.progress = wd.tick
    if getattr(args, "prep_in_worker", False):
        if rank == 0:
            prepare_data(args)
        comm.barrier()
    sess = make_session(args, comm, dev)
    if wd is not None:
        wd.logger = sess.bob_log if rank == 0 else None
        sess.timer.beacon = wd.beat
        wd.beat("session_ready")
    if args.resume_dir:
        sess.load_checkpoints(args.resume_dir)
    out = run_schedule(sess, args)
    if args.save_dir:
        sess.save_checkpoints(args.save_dir)
    if rank == 0:
        extra = {"mode": args.mode, "world_size": args.world_size, "nprocs": nprocs, "bob_tp": pl.bob_tp,
                 "device": str(dev), "kernels": ops.get_backend() if dev.type == "cuda" else "torch",
                 "last_eval": getattr(sess, "last_eval", None), "calib": getattr(args, "calib", None)}
        sess.timer.dump(os.path.join(args.log_dir, "metrics.json"), extra)
        if result_q is not None:
            result_q.put({"phases": out["phases"], **extra})
    sess.tracer.dump()
    if comm.msg_log is not None:
        with open(os.path.join(args.log_dir, f"messages_rank{rank}.json"), "w") as f:
            json.dump(comm.msg_log, f)
    sess.close()
    if wd is not None:
        wd.stop()
    if nprocs > 1:
        import torch.distributed as dist
        comm.barrier()
        dist.destroy_process_group()
    return out


def _spawn_entry(rank, nprocs, args):
    worker(rank, nprocs, args)


def launch(args):
    """Run the whole job (all ranks). Returns rank 0's metrics dict when run here."""
    env_rank = os.environ.get("RANK")
    if env_rank is not None and os.environ.get("WORLD_SIZE"):
        args.nprocs = int(os.environ["WORLD_SIZE"])
        args.master_addr = os.environ.get("MASTER_ADDR", args.master_addr)
        args.master_port = int(os.environ.get("MASTER_PORT", args.master_port))
        return worker(int(env_rank), args.nprocs, args)
    if args.nprocs == 1:
        return worker(0, 1, args)
    import torch.multiprocessing as mp
    mp.spawn(_spawn_entry, args=(args.nprocs, args), nprocs=args.nprocs, join=True)
    path = os.path.join(args.log_dir, "metrics.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def prepare_data(args, verbose=True):
    from ..data.mnist import shards_exist, write_shards
    if args.reuse_data and shards_exist(args.datapath, args.client_num_in_total):
        return
    write_shards(args, verbose=verbose, layout=getattr(args, "data_layout", "image"))


def main(argv=None):
    raise_fd_limit()
    args = resolve(parse_args(argv))
    os.makedirs(args.log_dir, exist_ok=True)           # Q15: loggers write here
    if os.environ.get("RANK") is not None and os.environ.get("WORLD_SIZE"):
        args.prep_in_worker = True                       # torchrun: rank 0 writes, then a barrier
    else:
        resolve_job_seed(args)                           # checkpointed jobs: record / reuse the seed
        prepare_data(args)                               # split_nn.py:179 (every run, Q12)
    if os.environ.get("RANK", "0") == "0":
        print("Initialize Meetup Spot", flush=True)
    return launch(args)


if __name__ == "__main__":
    main()
    sys.exit(0)
