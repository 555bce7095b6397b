"""The native split epoch of a REMOTE Alice (csrc/split.cpp roles 1 / 2 over the peer-mapped
channel, csrc/ipc_p2p.h) against the Python loop of the same placement: two real processes
on ONE GPU, Bob on rank 0 (one shard), Alice_1 on rank 1 (the BASELINE ws = 2 topology of
config 2, one process per role like the reference's mp.spawn).

    python scripts/split_remote_one_gpu.py vanilla|ushape B

Each rank builds two sessions with the same seed (one native, one `--python_epoch`), runs
two epochs over a shuffled order with a partial last batch, renews both optimizer slots
(the unlearn hand-off), runs one more epoch, and checks on its side: every parameter and
optimizer state bitwise equal between the two sessions, the step counts and Bob's dropout
counter equal, the per-batch message sequence (source, destination, bytes) equal, and the
channel's error word clear.  Each rank prints PASS.  Reference hot loops:
data_entities_vanilla.py:66-76, data_entities.py:65-81.
"""
import os
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _states(sess, kind):
    out = {}
    if sess.is_bob:
        for L in sess.tail.layers:
            out[f"bob.{L.spec.name}.W"] = L.W
            out[f"bob.{L.spec.name}.b"] = L.b
        for name, st in sess.bob_slot(1).states.items():
            for k, v in st.items():
                out[f"bobslot.{name}.{k}"] = v
    a = sess.alices.get(1)
    if a is not None:
        w, b = a.front.params
        out["front.w"], out["front.b"] = w, b
        if kind == "ushape":
            out["head.W"], out["head.b"] = a.head.layers[0].W, a.head.layers[0].b
        for name, st in a.slot.states.items():
            for k, v in st.items():
                out[f"aslot.{name}.{k}"] = v
    return out


def _data_msgs(log):
    """(src, dst, bytes) of the per-batch data messages, in issue order (the role agreement's
    one-int exchange excluded)."""
    return [(s, d, nb) for op, s, d, nb in log if op != "exchange" and nb > 64]


def worker(rank, world, port, kind, B, root):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # SL_RANK_DEVICES=D: rank r on cuda:(r % D) (tests/test_multi_gpu.py: the same protocol across
    # devices, over xGMI); default 1: every rank shares cuda:0
    ndev = int(os.environ.get("SL_RANK_DEVICES", "1"))
    torch.cuda.set_device(rank % ndev)
    dev = torch.device("cuda", rank % ndev)
    from splitlearning_amd import ops
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import UShapeSession, VanillaSession
    from splitlearning_amd.protocols.split_native import native_remote_role
    ops.set_backend("hip")
    data = os.path.join(root, "d")

    def make(native):
        flags = (["--vanilla"] if kind == "vanilla" else []) + ([] if native else ["--python_epoch"])
        args = parse_args(flags + ["--world_size", "2", "--seed", "11", "--num_samples", "1200", "--no_tqdm",
                                   "--batch_size", str(B), "--datapath", data, "--torch_p2p",
                                   "--log_dir", os.path.join(root, f"logs{rank}{int(native)}")])
        if rank == 0 and not os.path.exists(data):
            write_shards(args, verbose=False)
        dist.barrier()
        comm = Comm(rank, world, dev, Placement.make(2, 2, 1))
        comm.host_staging = True          # the Python loop's messages: staged through gloo
        comm.msg_log = []
        cls = VanillaSession if kind == "vanilla" else UShapeSession
        return cls(args, comm, dev)

    sp, sn = make(False), make(True)
    ok = sn.split_channel is not None and hasattr(sn.split_channel, "host_error")
    print(f"rank {rank}: peer-mapped split channel {'up' if ok else 'unavailable'}", flush=True)
    if ok:
        role = native_remote_role(sn, 1, kind)
        ok = role == ("bob" if rank == 0 else "alice") and native_remote_role(sp, 1, kind) is None
        print(f"rank {rank}: native role {role}", flush=True)
    if ok:
        n = min(B * 6 + 3, sn.n_train[1])
        gen = torch.Generator().manual_seed(4)
        order = sp.alices[1].train.shuffled_order(gen)[:n].to(dev) if rank == 1 else None
        for s in (sp, sn):
            s.comm.msg_log.clear()
        for _ in range(2):
            for s in (sp, sn):
                s.split_epoch(1, order, n)
        for s in (sp, sn):                    # the unlearn hand-off: fresh client + Bob slots
            if rank == 1:
                s.alices[1].slot = type(s.alices[1].slot)(s.alice_optim())
            else:
                s.bob_slots[1] = type(s.bob_slots[1])(s.bob_optim())
            s.split_epoch(1, order[:B * 3] if order is not None else None, B * 3)
        torch.cuda.synchronize()
        a, b = _states(sp, kind), _states(sn, kind)
        same = a.keys() == b.keys() and all(torch.equal(a[k], b[k]) for k in a)
        bad = [k for k in a if k in b and not torch.equal(a[k], b[k])]
        print(f"rank {rank}: {len(a)} tensors bitwise equal to the Python loop: {same} {bad[:4]}", flush=True)
        if rank == 1:
            same = same and sp.alices[1].slot.t == sn.alices[1].slot.t
            if kind == "ushape":
                same = same and sp.alices[1].head.fwd_count == sn.alices[1].head.fwd_count
        else:
            same = same and sp.bob_slot(1).t == sn.bob_slot(1).t and sp.tail.fwd_count == sn.tail.fwd_count
        mp_, mn = _data_msgs(sp.comm.msg_log), _data_msgs(sn.comm.msg_log)
        seq = mp_ == mn and len(mn) > 0
        print(f"rank {rank}: step counts equal {same}; message sequence equal {seq} "
              f"({len(mn)} sends, first {mn[:2]})", flush=True)
        err = sn.split_channel.error()
        print(f"rank {rank}: channel error word {err}", flush=True)
        ok = same and seq and err == 0
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    sp.close()
    sn.close()
    dist.destroy_process_group()
    if not all(flags):
        sys.exit(1)
    print(f"rank {rank}: PASS", flush=True)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "vanilla"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    port = 29700 + (os.getpid() % 1000)
    with tempfile.TemporaryDirectory() as root:
        mp.spawn(worker, args=(2, port, kind, B, root), nprocs=2, join=True)


if __name__ == "__main__":
    main()
