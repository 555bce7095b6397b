"""Session: the per-process runtime that hosts Bob (or a TP shard of him) and the
locally placed Alices, plus the request/response machinery shared by every mode.

The reference's role classes (`alice`/`bob` in data_entities*.py) talk through
RPC.  Here the same *method names* exist on the session, but each
is an SPMD-collective step: all processes call it in the same order (the Bob
schedule, `protocols/schedule.py`) and only the ranks hosting the involved roles
compute or move data.  Mode-specific behaviour lives in the subclasses
(vanilla.py, ushape.py, sisa.py, concat.py).
"""
from __future__ import annotations

import os
import random
from collections import Counter

import torch

from .. import ops
from ..config import CUT_FEATURES
from ..data.device_dataset import DeviceShard
from ..data.mnist import load_shard
from ..engine.front import FrontEngine
from ..engine.slots import OptSlot
from ..engine.tail import TailEngine
from ..parallel.dist import Comm, Placement
from ..utils.logging import NULL, role_logger
from ..utils.metrics import PhaseTimer
from ..utils.trace import make_tracer


def _progress(it, enabled, **kw):
    if not enabled:
        return it
    from tqdm import tqdm
    return tqdm(it, **kw)


class AliceState:
    """Everything one client owns (hosted on `placement.alice_rank(cid)`)."""

    def __init__(self, cid: int, logger, train: DeviceShard, test: DeviceShard, front: FrontEngine,
                 slot: OptSlot, gen: torch.Generator):
        self.cid = cid
        self.logger = logger
        self.train = train
        self.test = test
        self.front = front
        self.head: TailEngine | None = None
        self.slot = slot
        self.gen = gen
        self.unlearn_order: torch.Tensor | None = None


class Session:
    mode = "base"

    def __init__(self, args, comm: Comm, device: torch.device):
        self.args = args
        self.comm = comm
        self.pl: Placement = comm.pl
        self.rank = comm.rank
        self.device = device
        self.ops = ops.impl(device)
        # compute dtype of the GEMM-shaped kernels (process-wide switch of the op set)
        self.ops.set_compute_dtype(getattr(args, "dtype", "fp32"))
        self.k = args.client_num_in_total
        self.B = args.batch_size
        self.show = (not args.no_tqdm) and self.rank == 0
        # one agreed seed for everything that must match across ranks
        seed = args.seed if args.seed is not None else random.SystemRandom().randrange(1 << 62)
        self.seed = int(comm.broadcast_obj(seed, 0))
        self.bob_log = role_logger("bob", args.log_dir, self.rank == 0)
        self.timer = PhaseTimer(device, self.bob_log if self.rank == 0 else None, comm.barrier)
        self.tracer = make_tracer(args, self.rank, device)
        self.timer.tracer = comm.tracer = self.tracer
        self.alices: dict[int, AliceState] = {}
        self._build_alices()
        self._exchange_meta()
        self.is_bob = self.pl.is_bob(self.rank)
        self._native_data_plane()                          # collective over all ranks
        self.split_channel = self._split_channel()        # collective over all ranks
        self.tp_allreduce = self._tp_allreduce()          # collective over all ranks
        self.timer.check = self._check_transport
        self.tail: TailEngine | None = None
        self.bob_slots: dict = {}
        self.last_alice_id = None
        self.activation_and_labels_cache: dict = {}
        if self.is_bob:
            self._build_bob()
        self._resident_ok = self._decide_resident()       # collective over all ranks
        self.bob_log.info("Bob Started Getting Tipsy")
        if self.pl.bob_tp > 1:
            kind = ("peer-mapped (one kernel, fused into the server head)" if getattr(self, "tp_ipc", None) is not None
                    else "RCCL" if getattr(self, "tp_native_comm", None) is not None else "torch.distributed")
            self.bob_log.info(f"[perf] Bob tensor-parallel over {self.pl.bob_tp} ranks; TP all-reduce: {kind}")

    # ------------------------------------------------------------------ construction
    def _decide_resident(self) -> bool:
        """Whether Bob's epochs run on the register-resident executor (SISA overrides; a
        collective when it does, so every rank calls it)."""
        return False

    def front_module(self):
        from ..models import ClientFrontSisa
        return ClientFrontSisa()

    def alice_optim(self):
        raise NotImplementedError

    def bob_module_and_spec(self):
        raise NotImplementedError

    def bob_optim(self):
        raise NotImplementedError

    def _build_alices(self):
        for cid in self.pl.local_alices(self.rank):
            lg = role_logger(f"alice{cid}", self.args.log_dir, True)
            lg.info("Alice is going insane!")
            torch.manual_seed(self.seed + 1000 + cid)
            front = FrontEngine(self.front_module(), self.device)
            tr, te = self._load_client_shard(cid)
            train = DeviceShard(tr["x"], tr["y"], self.device)
            test = DeviceShard(te["x"], te["y"], self.device)
            gen = torch.Generator().manual_seed(self.seed + 7919 * cid)
            a = AliceState(cid, lg, train, test, front, OptSlot(self.alice_optim()), gen)
            self._extend_alice(a)
            self.alices[cid] = a
            lg.info("Local Data Statistics:")
            lg.info("Dataset Size: {:.2f}".format(train.n))
            lg.info("Training dataset: {}".format(train.label_counter()))
            lg.info("Test dataset: {}".format(test.label_counter()))

    def _extend_alice(self, a: AliceState):
        pass

    def _load_client_shard(self, cid: int):
        """`alice.load_data` (data_entities_vanilla_sisa.py:170-178): the client's
        tensor-only shard files.  Benchmarks override this with in-memory synthetic shards."""
        return load_shard(self.args.datapath, cid)

    def reset_activation_cache(self):
        self.activation_and_labels_cache.clear()
        if hasattr(self, "_ck"):
            self._ck.clear()

    def _exchange_meta(self):
        mine = {cid: (a.train.n, a.test.n) for cid, a in self.alices.items()}
        merged = {}
        for d in self._allgather_obj(mine):
            merged.update(d)
        self.n_train = {c: merged[c][0] for c in merged}
        self.n_test = {c: merged[c][1] for c in merged}

    def _allgather_obj(self, obj):
        if not self.comm.distributed:
            return [obj]
        import torch.distributed as dist
        out = [None] * self.comm.world
        dist.all_gather_object(out, obj)
        return out

    def _native_data_plane(self):
        """GPU, several processes: every p2p transfer (per-batch activation + labels, cut
        gradients, weight relay, SISA dump, eval traffic) through a native RCCL communicator
        over all ranks, issued on the compute stream (parallel/dist.py Comm.native)."""
        if (self.device.type == "cuda" and self.comm.distributed and self.comm.native is None
                and getattr(self.args, "native_comm", True)):
            from ..parallel.rccl import make_native_comm
            self.comm.native = make_native_comm(list(range(self.comm.world)), self.rank)

    def _split_channel(self):
        """The native split epoch's per-batch link for Alices remote from a one-shard Bob
        (vanilla / U-shape; protocols/split_native.py): the peer-mapped channel
        (`--split_channel auto|ipc`, csrc/ipc_p2p.h) or the RCCL communicator over all ranks.
        None when no such placement exists or no link could be set up (the Python loop then
        moves the messages)."""
        if self.mode not in ("vanilla", "ushape") or self.device.type != "cuda" or not self.comm.distributed:
            return None
        if self.pl.bob_tp != 1 or all(r == self.pl.bob_root for r in self.pl.alice_ranks.values()):
            return None
        kind = getattr(self.args, "split_channel", "auto")
        if kind in ("auto", "ipc"):
            from ..parallel.rccl import make_ipc_channel
            ch = make_ipc_channel(self.packed_len(self.B, torch.float32))
            if ch is not None or kind == "ipc":
                return ch
        return self.comm.native

    def _tp_allreduce(self):
        """Bob's TP all-reduce: a native RCCL communicator on GPUs (capturable in the
        server-step graph), the torch.distributed group otherwise (gloo on CPU)."""
        if self.pl.bob_tp <= 1:
            return self.comm.tp_allreduce
        if self.device.type == "cuda" and getattr(self.args, "native_comm", True):
            from ..parallel.rccl import make_native_comm, native_allreduce
            tpc = make_native_comm(self.pl.bob_ranks, self.rank)
            self.tp_native_comm = tpc
            self.tp_ipc = None
            if tpc is not None and getattr(self.args, "tp_allreduce", "auto") == "auto":
                # one-kernel all-reduce over peer-mapped HBM for the per-step fc2 partial;
                # RCCL keeps every larger message and any rank set where set-up or the
                # self-test fails (decided together)
                from ..parallel.rccl import make_ipc_allreduce
                self.tp_ipc = make_ipc_allreduce(self.pl.bob_ranks, self.rank)
                if self.tp_ipc is not None:
                    tpc.attach_ipc(self.tp_ipc)
            if tpc is None and getattr(self.args, "tp_allreduce", "auto") == "auto":
                # no RCCL communicator (ranks sharing one GPU): the peer-mapped all-reduce alone
                from ..parallel.rccl import ipc_allreduce, make_ipc_allreduce
                self.tp_ipc = make_ipc_allreduce(self.pl.bob_ranks, self.rank)
                if self.tp_ipc is not None:
                    return ipc_allreduce(self.tp_ipc)
            if tpc is None:
                return self.comm.tp_allreduce
            ar = native_allreduce(tpc)
            if self.tp_ipc is not None:
                ar.ipc = self.tp_ipc     # the register-resident epoch exchanges through it in-launch
            return ar
        return self.comm.tp_allreduce

    def _check_transport(self):
        """Phase-end check (after the device sync): the peer-mapped all-reduce's bounded waits
        raise an error word instead of hanging; a phase that hit one fails loudly here."""
        ch = getattr(self, "split_channel", None)
        if ch is not None and hasattr(ch, "host_error") and ch.error() != 0:
            raise RuntimeError("peer-mapped split channel: a message wait timed out on this rank (the peer "
                               "stalled or the mapping is broken); rerun with --split_channel rccl")
        ipc = getattr(self, "tp_ipc", None)
        if ipc is not None and ipc.error() != 0:
            raise RuntimeError("peer-mapped TP all-reduce: a flag wait timed out on this rank (a peer "
                               "stalled or the mapping is broken); rerun with --tp_allreduce rccl")

    def _build_bob(self):
        module, spec = self.bob_module_and_spec()
        tp_size = self.pl.bob_tp
        tp_rank = self.pl.bob_ranks.index(self.rank)
        self.tail = TailEngine(module, spec, self.device, tp_rank, tp_size,
                               allreduce=self.tp_allreduce, seed_base=self.seed)
        if getattr(self.comm, "host_staging", False) and tp_size > 1:
            # Bob's TP ranks share ONE GPU (the --ranks_share_gpu rehearsal): each persistent
            # launch takes its share of the CUs so all of them are resident together
            self.tail.resident_workgroups = max(8, (256 // tp_size) // 8 * 8)

    def make_bob_module(self, cls, *a):
        # identical init on every TP rank: seed the default generator with the agreed seed
        torch.manual_seed(self.seed + 17)
        return cls(*a)

    # ------------------------------------------------------------------ placement helpers
    def host(self, cid: int) -> int:
        return self.pl.alice_rank(cid)

    def hosts(self, cid: int) -> bool:
        return cid in self.alices

    @property
    def bob_ranks(self):
        return self.pl.bob_ranks

    def to_bob(self, cid: int, t, shape, dtype=torch.float32):
        """Alice_cid -> every Bob TP rank."""
        return self.comm.multicast(t, self.host(cid), self.bob_ranks, shape, dtype)

    def from_bob(self, cid: int, t, shape, dtype=torch.float32):
        """Bob (root TP rank; the value is replicated) -> Alice_cid."""
        out = self.comm.send_recv(t if self.rank == self.pl.bob_root else None, self.pl.bob_root,
                                  self.host(cid), shape, dtype)
        if self.hosts(cid) and self.rank == self.pl.bob_root:
            return t
        return out

    def split_lookahead(self, cid: int) -> bool:
        """Whether a split-mode epoch of Alice_cid uses Bob's fc1 look-ahead (Bob's update of
        batch i is issued after Alice's forward of batch i+1, so its kernel also forms that
        batch's fc1 product and Bob never re-reads fc1 for a forward) — or the §3.2 overlap
        order (Bob's update issued right after the cut gradient leaves, so it runs while the
        Alice does her backward and next forward; Bob then re-reads fc1 for that forward).

        Placement decides (docs/ARCHITECTURE.md, "Split-mode schedule"): when the Alice's GPU
        runs a Bob shard (one GPU; Bob tensor-parallel over every GPU, the vanilla default)
        her work and that shard's update share one stream, so the overlap order moves nothing
        off the critical path and only adds fc1's forward read back: look-ahead.  When no Bob
        shard lives on her GPU (U-shape's TP = 1 policy on several GPUs, or `--bob_tp` < N)
        the update of batch i can hide behind her step: overlap order."""
        return self.host(cid) in self.bob_ranks

    @property
    def act_dtype(self):
        """Wire / cache dtype of cut-layer activations (`--act_dtype`): bf16 halves every
        activation transfer (and SISA's cache); compute stays fp32."""
        return torch.bfloat16 if getattr(self.args, "act_dtype", "fp32") == "bf16" else torch.float32

    def act_to_bob(self, cid: int, act, B: int):
        """Cut activation [B, cut] Alice_cid -> every Bob rank in the wire dtype, fp32 on arrival.
        With a bf16 wire the host rounds its own copy too, so every Bob rank (and every
        placement of the roles) sees the same input."""
        wire = self.act_dtype
        if wire != torch.float32 and act is not None:
            act = act.to(wire)
        got = self.to_bob(cid, act, (B, self.cut_width_in()), wire)
        return got.float() if (got is not None and wire != torch.float32) else got

    def to_bob_var(self, cid: int, t, inner_shape, dtype):
        """Variable-length Alice -> Bob transfer (length header first)."""
        n = torch.tensor([t.shape[0] if t is not None else 0], dtype=torch.int64, device=self.device)
        n = self.to_bob(cid, n if self.hosts(cid) else None, (1,), torch.int64)
        if n is None:
            return None
        rows = int(n.item())
        return self.to_bob(cid, t, (rows,) + tuple(inner_shape), dtype)

    @staticmethod
    def packed_len(B: int, dtype) -> int:
        """Elements of one packed [activation | labels] message in the wire dtype: the labels
        ride as int64 words behind the rows, the whole padded to 16-byte units (the layout the
        native split executor sends too, csrc/split.cpp act_msg_words)."""
        es = torch.empty((), dtype=dtype).element_size()
        n = B * CUT_FEATURES + B * (8 // es)
        unit = 16 // es
        return -(-n // unit) * unit

    @classmethod
    def pack(cls, act: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """One message per batch: [B*5408 activation | B int64 labels] in the activation's
        dtype (labels bit-exact whatever the wire dtype)."""
        B = act.shape[0]
        buf = torch.zeros(cls.packed_len(B, act.dtype), device=act.device, dtype=act.dtype)
        buf[:B * CUT_FEATURES].view(B, CUT_FEATURES).copy_(act)
        per = 8 // act.element_size()
        buf[B * CUT_FEATURES:B * CUT_FEATURES + B * per].view(torch.int64).copy_(labels)
        return buf

    @staticmethod
    def unpack(buf: torch.Tensor, B: int):
        act = buf[:B * CUT_FEATURES].view(B, CUT_FEATURES)
        per = 8 // buf.element_size()
        labels = buf[B * CUT_FEATURES:B * CUT_FEATURES + B * per].view(torch.int64)
        return act, labels

    def send_act_labels(self, cid, act, labels, B):
        """Cut activation + labels Alice -> Bob, packed into one message when remote."""
        host = self.host(cid)
        wire = self.act_dtype
        if wire != torch.float32 and act is not None:
            act = act.to(wire).float()             # every Bob rank sees the rounded input
        remote = [r for r in self.bob_ranks if r != host]
        if not remote:
            return (act, labels) if self.is_bob else (None, None)
        pkt = self.pack(act.to(wire), labels) if self.rank == host else None
        got = self.comm.multicast(pkt, host, self.bob_ranks, (self.packed_len(B, wire),), wire)
        if not self.is_bob:
            return None, None
        if self.rank == host:
            return act, labels
        a, lab = self.unpack(got, B)
        return a.float(), lab

    # ------------------------------------------------------------------ shared Alice API
    def give_weights(self, cid: int) -> dict:
        """Reference `alice.give_weights` (data_entities_vanilla.py:79-80): a copy of the
        client's state_dict (reference key names)."""
        a = self.alices[cid]
        return {k: v.detach().clone() for k, v in a.front.module.state_dict().items()}

    def relay_weights(self, src_cid: int, dst_cid: int):
        """Round-robin "Snapshot" hand-off Alice_src -> Alice_dst (M5): one flat buffer, p2p."""
        s, d = self.host(src_cid), self.host(dst_cid)
        if self.rank not in (s, d):
            return
        if s == d:
            flat = self._flat_client_weights(self.alices[src_cid])
            self._load_flat_client_weights(self.alices[dst_cid], flat)
            return
        n = self._client_flat_numel()
        t = self._flat_client_weights(self.alices[src_cid]) if self.rank == s else None
        got = self.comm.send_recv(t, s, d, (n,), torch.float32)
        if self.rank == d:
            self._load_flat_client_weights(self.alices[dst_cid], got)

    def _flat_client_weights(self, a: AliceState) -> torch.Tensor:
        return a.front.flat_weights()

    def _load_flat_client_weights(self, a: AliceState, flat):
        a.front.load_flat_weights(flat)

    def _client_flat_numel(self) -> int:
        return 32 * 9 + 32

    def freeze_alice_weights(self, client_ids):
        for cid in client_ids:
            self.bob_log.info("Server training starts. Freezing weights for Alices-{}.".format(cid))
            if self.hosts(cid):
                self.alices[cid].front.frozen = True

    def unfreeze_alice_weights(self, client_ids):
        for cid in client_ids:
            self.bob_log.info("Unfreezing weights for Alices-{}.".format(cid))
            if self.hosts(cid):
                self.alices[cid].front.frozen = False

    def switch_mode_to_train(self):
        if self.tail is not None:
            self.tail.training = True

    def switch_mode_to_eval(self):
        if self.tail is not None:
            self.tail.training = False

    def reset_model(self, cid: int):
        self.alices[cid].front.reset_parameters(self.args.true_reset)

    def unlearn_samples(self, cid: int) -> int:
        """Collective: the size of Alice_cid's unlearn (label-filtered) training set, known
        on her host rank, agreed by every rank (phase sample counts)."""
        a = self.alices.get(cid)
        n = int(a.unlearn_order.numel()) if (a is not None and a.unlearn_order is not None) else 0
        if not self.comm.distributed:
            return n
        return int(self.comm.broadcast_obj(n, self.host(cid)))

    def filtered_order(self, a: AliceState, omit_label: int) -> torch.Tensor:
        """`[(x, y) for batch in train_dataloader for x, y in zip(*batch) if y != omit]`:
        one shuffled pass over the shard with the omitted label dropped."""
        return a.train.filtered_order(a.train.shuffled_order(a.gen), omit_label)

    # ------------------------------------------------------------------ evaluation
    def _bob_logits_for(self, cid: int, act):
        """Bob's inference on Alice_cid's activations; logits delivered to Alice_cid."""
        n = self.n_test[cid]
        act_b = self.act_to_bob(cid, act, n)
        out = None
        if self.is_bob:
            out = self.bob_infer(act_b, cid)
        return self.from_bob(cid, out, (n, self.bob_out_width()), torch.float32)

    def cut_width_in(self) -> int:
        return CUT_FEATURES

    def bob_out_width(self) -> int:
        return self.tail.spec.out_features if self.tail is not None else 100

    def bob_infer(self, act, cid):
        return self.tail.forward(act)

    def client_logits(self, cid: int, bob_out):
        return bob_out

    def _eval_counts(self, omit_label: int):
        """counters[k+1, 6] summed over ranks (row c = Alice_c)."""
        counts = torch.zeros(self.k + 1, 6, dtype=torch.int64, device=self.device)
        # every hosted Alice's test activations from one launch per chunk (frozen fronts)
        hosted = [cid for cid in range(1, self.k + 1) if self.hosts(cid)]
        acts = dict(zip(hosted, FrontEngine.forward_multi([self.alices[c].front for c in hosted],
                                                          [self.alices[c].test for c in hosted],
                                                          [None] * len(hosted))))
        for cid in range(1, self.k + 1):
            act = acts.pop(cid, None)
            logits = self._bob_logits_for(cid, act)
            if self.hosts(cid):
                a = self.alices[cid]
                logits = self.client_logits(cid, logits)
                counts[cid] = self.ops.eval_counters(logits, a.test.y, omit_label)
        self.comm.allreduce_sum_(counts)
        return counts.cpu()

    def eval_request(self):
        self.bob_log.info("Initializing Evaluation of all Alices")
        self.before_eval()
        c = self._eval_counts(-1)
        for cid, a in self.alices.items():
            corr, tot = int(c[cid, 0]), int(c[cid, 1])
            a.logger.info(f"Alice-{cid} Evaluating Data: {round(corr / tot if tot else 0, 3)}")
        corr, tot = int(c[1:, 0].sum()), int(c[1:, 1].sum())
        self.bob_log.info("Accuracy over all data: {:.3f}".format(corr / tot if tot else 0.0))
        return corr, tot

    def eval_request_breakdown(self, omit_label: int):
        self.bob_log.info("Initializing Evaluation of all Alices. Breaking down to the unlearned and the "
                          "remaining data")
        self.before_eval()
        c = self._eval_counts(omit_label)
        for cid, a in self.alices.items():
            corr, tot, cu, tu, cr, tr = (int(v) for v in c[cid])
            a.logger.info(f"Alice-{cid} Evaluating Data: {round(corr / tot if tot else 0, 3)}")
            a.logger.info(f"Alice-{cid} Evaluating Unlearned label-{omit_label}: "
                          f"{round(cu / tu if tu else 0, 3)}")
            a.logger.info(f"Alice-{cid} Evaluating Remaining labels: {round(cr / tr if tr else 0, 3)}")
        s = c[1:].sum(0).tolist()
        # Q14: the reference divides by zero when no test sample carries the omitted label
        self.bob_log.info("Accuracy over all data: {:.3f}".format(s[0] / s[1] if s[1] else 0.0))
        self.bob_log.info("Accuracy over unlearned data: {:.3f}".format(s[2] / s[3] if s[3] else 0.0))
        self.bob_log.info("Accuracy over remaining data: {:.3f}".format(s[4] / s[5] if s[5] else 0.0))
        self.last_eval = s
        return s

    def before_eval(self):
        pass

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoints(self, out_dir: str):
        """Reference-layout state_dicts: bob.pt (full, gathered from TP shards) and
        alice{c}.pt.  Loadable with torch.load(weights_only=True)."""
        os.makedirs(out_dir, exist_ok=True)
        if self.is_bob:
            sd = self.tail.full_state_dict(self.comm.tp_allgather)
            if self.rank == self.pl.bob_root:
                torch.save(sd, os.path.join(out_dir, "bob.pt"))
        for cid, a in self.alices.items():
            torch.save(self._client_state(a), os.path.join(out_dir, f"alice{cid}.pt"))
        self.comm.barrier()

    def _client_state(self, a: AliceState) -> dict:
        return {k: v.detach().cpu() for k, v in a.front.module.state_dict().items()}

    def load_checkpoints(self, in_dir: str):
        if self.is_bob:
            sd = torch.load(os.path.join(in_dir, "bob.pt"), weights_only=True)
            self.tail.load_full_state_dict(sd)
        for cid, a in self.alices.items():
            sd = torch.load(os.path.join(in_dir, f"alice{cid}.pt"), weights_only=True)
            self._load_client_state(a, sd)
        self.comm.barrier()

    def _load_client_state(self, a: AliceState, sd: dict):
        a.front.module.load_state_dict({k: v.to(self.device) for k, v in sd.items()})

    # ------------------------------------------------------------------ misc
    def label_counter(self, a: AliceState, order) -> dict:
        return dict(Counter(a.train.y_cpu[order.cpu()].tolist()))

    def close(self):
        from ..utils.logging import close_all
        close_all(["bob"] + [f"alice{c}" for c in self.alices])


__all__ = ["Session", "AliceState", "NULL", "_progress"]
