"""A tensor-parallel Bob rank that dies mid-epoch must take the job down within one
peer-mapped wait timeout, not one timeout per remaining step.

T real processes on the box's one GPU each run their shard of the production native
executor (`_C.ServerEpoch`) with the peer-mapped all-reduce (csrc/ipc_ar.h) between them.
Rank T-1 runs only the first `stop` steps of the epoch and then stops issuing work (a
stalled peer; it sleeps, and the launcher kills it once the survivors are gone).  Every
surviving rank's fused head waits for the dead rank's flags, times out once (`--timeout`),
raises the error word, and every later wait gives up at once; `ServerEpoch::run` reads the
host-pinned mirror of the word every 64 steps without a device sync and raises.  Each
survivor prints the seconds from the peer's death to its abort and exits 3.

    python scripts/tp_peer_failure_one_gpu.py [T] [timeout_s]
Reference: a child failure ends the job (split_nn.py:183-186, mp.spawn join=True).
"""
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, timeout_s, stamp):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from splitlearning_amd import ops
    from splitlearning_amd.engine import OptSlot, TailEngine, adam
    from splitlearning_amd.models import ServerTailSisa, sisa_server_spec
    from splitlearning_amd.parallel.rccl import ipc_allreduce, make_ipc_allreduce
    ops.set_backend("hip")
    ipc = make_ipc_allreduce(list(range(world)), rank)
    if ipc is None:
        print(f"rank {rank}: ipc allreduce unavailable", flush=True)
        sys.exit(2)
    ipc.set_timeout_s(timeout_s)
    B, steps, stop = 16, 1200, 40
    g = torch.Generator().manual_seed(5)
    acts = (torch.rand(B * steps, 5408, generator=g) * 30).to(dev)
    labels = torch.randint(0, 10, (B * steps,), generator=g).to(dev)
    torch.manual_seed(0)
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=rank, tp_size=world,
                      allreduce=ipc_allreduce(ipc), seed_base=3)
    slot = OptSlot(adam(1e-3, 1e-5))
    dist.barrier()
    tail.lookahead_prologue(acts[:B])
    if rank == world - 1:
        tail.run_native_epoch(acts[:B * stop].contiguous(), labels[:B * stop].contiguous(), slot, B, True)
        torch.cuda.synchronize()
        with open(stamp, "w") as f:
            f.write(repr(time.time()))
        print(f"rank {rank}: ran {stop} steps, stalling", flush=True)
        time.sleep(60)
        os._exit(9)
    try:
        tail.run_native_epoch(acts, labels, slot, B, True)
        torch.cuda.synchronize()
        err = ipc.error()
        if err:
            raise RuntimeError("peer-mapped TP all-reduce error word set")
        print(f"rank {rank}: epoch finished without noticing the dead peer", flush=True)
        os._exit(0)
    except RuntimeError as e:
        t = time.time()
        for _ in range(100):
            if os.path.exists(stamp):
                break
            time.sleep(0.05)
        t0 = float(open(stamp).read()) if os.path.exists(stamp) else float("nan")
        with open(f"{stamp}.r{rank}", "w") as f:
            f.write(repr(t - t0))
        print(f"rank {rank}: aborted {t - t0:.2f} s after the peer stalled: {str(e).splitlines()[0]}", flush=True)
        os._exit(3)


if __name__ == "__main__":
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    tmo = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    stamp = f"/tmp/sl_peer_dead_{os.getpid()}"
    if os.path.exists(stamp):
        os.remove(stamp)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r, T, 29711 + T, tmo, stamp)) for r in range(T)]
    t0 = time.time()
    for p in procs:
        p.start()
    for p in procs[:-1]:
        p.join(timeout=90)
    procs[-1].join(timeout=1)
    codes = []
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
        codes.append(p.exitcode)
    print(f"exit codes {codes} wall {time.time() - t0:.1f} s", flush=True)
    # every survivor aborted, within twice the wait timeout of the stall (not timeout x steps)
    lat = []
    for r in range(T - 1):
        f = f"{stamp}.r{r}"
        lat.append(float(open(f).read()) if os.path.exists(f) else float("inf"))
    print(f"abort latency after the stall, s: {[round(v, 2) for v in lat]} (bound {2 * tmo:.1f})", flush=True)
    ok = codes[-1] != 0 and all(c == 3 for c in codes[:-1]) and all(v < 2 * tmo for v in lat)
    print("PASS" if ok else "FAIL", flush=True)
    sys.exit(0 if ok else 1)
