"""SISA split learning + unlearning (`--sisa`) and the retrain-from-scratch
control group (`--control`).

Reference: `/root/reference/data_entities_vanilla_sisa.py` (alice `:35-250`,
bob `:253-419`), schedules `split_nn.py:74-117` (SISA) and `:119-135` (control;
the reference routes `--control` to the wrong module and crashes, Q2 — here it
gets the SISA semantics its methods were written for).

Phases and their MI355X mapping:
* local training — every Alice trains her conv front alone (CE on the 5408-wide
  activation, Q5; Adam wd=1e-5), all Alices concurrently, one per GPU, each
  batch = 3 kernels (gather+conv, softmax-CE, conv-backward+Adam), zero comm;
* activation dump — on first use per cache key `(client, unlearned, unlearn_id)`
  the client's whole shard goes through the frozen front and the activations +
  labels are multicast p2p to every Bob TP rank, where they stay resident in HBM
  (`activation_and_labels_cache`, SISA's isolated-slice cache, Q17);
* server training — Bob's Adam(wd=1e-5) epochs over the cached activations, no
  communication except the TP all-reduce inside each step;
* unlearning — only the requesting Alice retrains (without the omitted label);
  only her cache entry is recomputed; Bob retrains on top of his current weights.
"""
from __future__ import annotations

import torch

from ..config import ADAM_WEIGHT_DECAY, CUT_FEATURES
from ..engine.front import FrontEngine
from ..engine.slots import OptSlot, adam
from ..models import ServerTailSisa, sisa_server_spec
from .base import AliceState, Session, _progress


def executor_wants(args):
    """(resident, hybrid) wants for engine/resident.decide from the CLI: `--resident` and
    `--hybrid` gate their own executor only; both persistent executors compute in fp32, so
    `--dtype bf16` turns both off with that reason (reported as `server_executor_reason`)."""
    if getattr(args, "dtype", "fp32") != "fp32":
        why = f"dtype {args.dtype}: the persistent executors compute in fp32 only"
        return why, why
    return getattr(args, "resident", "auto") != "off", getattr(args, "hybrid", "auto") != "off"


class SisaSession(Session):
    mode = "sisa"

    def alice_optim(self):
        return adam(self.args.lr, ADAM_WEIGHT_DECAY)

    def bob_optim(self):
        return adam(self.args.lr, ADAM_WEIGHT_DECAY)

    def bob_module_and_spec(self):
        return self.make_bob_module(ServerTailSisa), sisa_server_spec()

    def _build_bob(self):
        super()._build_bob()
        self.bob_slots["server"] = OptSlot(self.bob_optim())

    @property
    def bob_slot(self) -> OptSlot:
        return self.bob_slots["server"]

    def before_eval(self):
        # each reference Alice calls bob.switch_mode_to_eval() before evaluating
        self.switch_mode_to_eval()

    # ------------------------------------------------------------------ Alice-local training
    def local_step(self, a: AliceState, idx):
        """`zero_grad; CE(model(x), y).backward(); step` (data_entities_vanilla_sisa.py:60-70)."""
        a.front.local_step(a.train, idx, a.slot)

    def local_train(self, a: AliceState, fixed_order=None):
        """`epochs` local epochs; reshuffled every epoch unless a fixed (unlearn /
        filtered, shuffle=False) order is given."""
        for _ in _progress(range(self.args.epochs), self.show, desc="Epochs", ascii=" >="):
            order = fixed_order if fixed_order is not None else a.train.shuffled_order(a.gen)
            with self.tracer.gpu_span(f"local_epoch[alice{a.cid}]", samples=int(order.numel())):
                a.front.local_epoch(a.train, order, self.B, a.slot)
            self.comm.progress()

    def train(self, cid: int):
        a = self.alices[cid]
        a.logger.info("Local Training")
        self.local_train(a)

    # ------------------------------------------------------------------ Bob API
    def train_request(self, client_id: int):
        self.bob_log.info(f"Train Request for Alice-{client_id}")
        if self.hosts(client_id):
            self.train(client_id)
        self.comm.barrier()

    def train_request_parallel(self):
        """Reference `bob.train_request_parallel` (data_entities_vanilla_sisa.py:326-334): every
        Alice trains at once.  Across processes they run concurrently anyway; the Alices
        co-located on this process are stepped together (`FrontEngine.local_epoch_multi`: one
        launch per step for all of them) instead of one epoch after another."""
        self.bob_log.info("Train all Alices in parallel")
        cids = sorted(self.alices)
        if len(cids) > 1 and getattr(self.args, "multi_alice", True):
            als = [self.alices[c] for c in cids]
            for a in als:
                a.logger.info("Local Training")
            for _ in _progress(range(self.args.epochs), self.show, desc="Epochs", ascii=" >="):
                orders = [a.train.shuffled_order(a.gen) for a in als]
                with self.tracer.gpu_span(f"local_epoch[alices{cids}]", samples=int(sum(o.numel() for o in orders))):
                    FrontEngine.local_epoch_multi([a.front for a in als], [a.train for a in als], orders, self.B,
                                                  [a.slot for a in als])
                self.comm.progress()
        else:
            for cid in cids:
                self.train(cid)
        self.comm.barrier()        # "wait for all futures"

    def train_request_control(self, client_id: int, omit_label: int):
        self.bob_log.info(f"Train Request for Alice-{client_id}")
        if self.hosts(client_id):
            self.train_control(client_id, omit_label)
        self.comm.barrier()

    def train_control(self, cid: int, omit_label: int):
        """Reference `alice.train_control` (data_entities_vanilla_sisa.py:230-250)."""
        a = self.alices[cid]
        order = self.filtered_order(a, omit_label)
        a.unlearn_order = order
        a.logger.info("Filtered dataset: {}".format(self.label_counter(a, order)))
        self.local_train(a, fixed_order=order)

    def unlearn_request(self, client_id: int, omit_label: int):
        self.bob_log.info(f"Unlearn Request for Alice-{client_id} upon the label-{omit_label}")
        if self.hosts(client_id):
            self.unlearn(client_id, omit_label)
        self.comm.barrier()

    def unlearn(self, cid: int, omit_label: int):
        """Reference `alice.unlearn` (data_entities_vanilla_sisa.py:139-168)."""
        a = self.alices[cid]
        a.logger.info(f"Unlearning label: {omit_label}, and reset the model")
        self.reset_model(cid)
        a.slot = OptSlot(self.alice_optim())
        order = self.filtered_order(a, omit_label)
        a.unlearn_order = order
        a.logger.info("Retraining dataset: {}".format(self.label_counter(a, order)))
        a.logger.info("Test dataset (retraining): {}".format(a.test.label_counter()))
        self.local_train(a, fixed_order=order)

    def give_activation_and_labels(self, cid: int, unlearned: bool = False):
        """Alice side of the dump: (activations [n,5408], labels [n]) over the train loader
        (fresh shuffle) or the unlearn loader (fixed order)."""
        return self._give_many([(cid, unlearned)])[cid]

    def _give_many(self, reqs) -> dict:
        """`give_activation_and_labels` of several hosted Alices [(cid, unlearned)]: their
        frozen fronts run together, one launch per chunk of rows (FrontEngine.forward_multi)."""
        fronts, shards, orders = [], [], []
        for cid, unlearned in reqs:
            a = self.alices[cid]
            if unlearned:
                if a.unlearn_order is None:
                    raise RuntimeError(f"Alice-{cid} has no unlearn dataloader (unlearn/train_control first)")
                order = a.unlearn_order
            else:
                order = a.train.shuffled_order(a.gen)
            fronts.append(a.front)
            shards.append(a.train)
            orders.append(order)
        out = {}
        for (cid, _), acts, order in zip(reqs, FrontEngine.forward_multi(fronts, shards, orders), orders):
            if self.act_dtype != torch.float32:
                acts = acts.to(self.act_dtype)
            out[cid] = (acts, self.alices[cid].train.y[order])
        return out

    def get_activation_and_labels(self, client_id: int, unlearned: bool = False, unlearn_id=None, dumped=None):
        key = (client_id, unlearned, unlearn_id)
        hit = self.activation_and_labels_cache.get(key) if self.is_bob else None
        # every rank must agree on hit/miss: the cache is replicated on all Bob ranks and
        # keys are inserted in schedule order, so a Bob-side membership test is enough —
        # non-Bob ranks track the key set too
        known = key in self._cache_keys
        if known:
            return hit
        acts = labels = None
        if self.hosts(client_id):
            acts, labels = dumped if dumped is not None else self.give_activation_and_labels(client_id, unlearned)
        acts = self.to_bob_var(client_id, acts, (CUT_FEATURES,), self.act_dtype)
        labels = self.to_bob_var(client_id, labels, (), torch.int64)
        self._cache_keys.add(key)
        if self.is_bob:
            self.activation_and_labels_cache[key] = (acts, labels)
            return acts, labels
        return None

    def prefetch_activations(self, unlearn_request_from_alices=(), unlearn_id=None):
        """Fill Bob's activation cache for every client in one batched transfer.

        The reference pulls the dumps one client at a time (rpc_sync per client,
        data_entities_vanilla_sisa.py:272-292, 299-302).  Here every host rank runs its
        Alices' frozen fronts first, then all (client -> Bob rank) transfers are posted as
        one batch of p2p ops, so N hosts stream into Bob's ranks over their own links at
        once.  Collective; cache keys are identical to
        `get_activation_and_labels`, which then hits."""
        keys = []
        for cid in range(1, self.k + 1):
            unl = cid in unlearn_request_from_alices
            key = (cid, unl, unlearn_id if unl else None)
            if key not in self._cache_keys:
                keys.append(key)
        if not keys:
            return
        dumps = self._give_many([(cid, unl) for cid, unl, _ in keys if self.hosts(cid)])
        if not self.comm.distributed:
            for cid, unl, uid in keys:
                self.get_activation_and_labels(cid, unlearned=unl, unlearn_id=uid, dumped=dumps.get(cid))
            return
        local = {}
        counts = torch.zeros(self.k + 1, dtype=torch.int64, device=self.device)
        for cid, (acts, labels) in dumps.items():
            local[cid] = self.pack(acts, labels)
            counts[cid] = labels.numel()
        self.comm.allreduce_sum_(counts)
        counts = counts.tolist()
        sends, recvs, got = [], [], {}
        for cid, _, _ in keys:
            n, h = counts[cid], self.host(cid)
            if self.rank == h:
                sends += [(local[cid], b) for b in self.bob_ranks if b != h]
                got[cid] = local[cid]
            elif self.is_bob:
                got[cid] = torch.empty(self.packed_len(n, self.act_dtype), device=self.device, dtype=self.act_dtype)
                recvs.append((got[cid], h))
        self.comm.exchange(sends, recvs)
        for key in keys:
            cid = key[0]
            self._cache_keys.add(key)
            if self.is_bob:
                self.activation_and_labels_cache[key] = self.unpack(got[cid], counts[cid])

    @property
    def _cache_keys(self) -> set:
        if not hasattr(self, "_ck"):
            self._ck = set()
        return self._ck

    def server_step(self, x, y, pre: bool = False, x_next=None):
        """`zero_grad; CE(model(x), y).backward(); step` on Bob (data_entities_vanilla_sisa.py:305-313).
        `pre` / `x_next`: the fc1 look-ahead chain (TailEngine.fused_step)."""
        if self.tail.fused3_ok():
            self.tail.train_fwd_bwd3(x, y, need_dx=False, pre=pre)
            self.tail.fused_step(self.bob_slot, x_next=x_next)
            return
        out = self.tail.forward(x, train=True)
        _, d = self.ops.softmax_ce(out, y, 1.0 / x.shape[0])
        self.tail.backward_dgrad(d, need_dx=False)
        self.tail.backward_step(self.bob_slot)

    GRAPH_STEPS = 16

    def _use_graphs(self) -> bool:
        mode = getattr(self.args, "graphs", "auto")
        if mode == "off" or self.device.type != "cuda":
            return False
        if mode == "auto" and getattr(self.args, "native_epoch", True) and self.tail.native_epoch_ok(self.B):
            # the native executor issues the same steps from C++ at ~17-25 us of host time
            # per step, and skips the graph's per-chunk staging copies (187.9 vs 190.0 us per
            # step at TP = 1, 54.4 vs 56.1 at TP = 8)
            return False
        if mode == "auto" and self.B > 128:
            # batches past the skinny kernels' range: eagerly the fp32 products go to
            # hipBLASLt, which cannot be captured (a graph would fall back to the in-tree
            # kernels: 299.7 k vs 386.6 k samples/s at batch 256 vs 128 captured)
            return False
        if self.tail.tp_size != 1:
            # A TP shard step is GPU-bound even eagerly (measured 58 us eager vs 59 us
            # replayed at TP=8, docs/PERF.md), so "auto" keeps the collective out of the
            # graph; "on" captures it when the all-reduce is the native RCCL communicator.
            if mode != "on" or not getattr(self.tail.allreduce, "capturable", False):
                return False
        from .. import ops as _ops
        return _ops.get_backend() != "torch"

    def _use_resident(self) -> bool:
        """Bob's server epochs on the register-resident executor (the whole shard on-chip)."""
        return getattr(self, "server_executor", "launch_per_stage") == "resident"

    def _use_hybrid(self) -> bool:
        """Bob's server epochs on the hybrid persistent executor (wide shard, fc1 streamed)."""
        return getattr(self, "server_executor", "launch_per_stage") == "hybrid"

    def _decide_resident(self) -> bool:
        """Collective over every rank (Session.__init__): which persistent executor, if any,
        runs Bob's server epochs (engine/resident.py decide: the register-resident epoch where
        the shard fits on-chip, else the hybrid epoch; tensor-parallel, only after every Bob
        rank's self-test passed with the same replicated fc3, otherwise the peer-mapped region
        is re-armed on every rank and Bob keeps the launch-per-stage executor).  The outcome
        and its reason land in `server_executor` / `resident_status` (bench JSON).  Returns
        whether the register-resident executor was adopted."""
        from ..engine import resident
        want, want_h = executor_wants(self.args)
        kind, why = resident.decide(self.tail if self.is_bob else None, self.bob_slot if self.is_bob else None,
                                    self.B, self.comm.distributed, want, want_h)
        self.server_executor = kind
        self.resident_status = {"executor": kind, "reason": why, "adopted": kind == "resident"}
        return kind == "resident"

    def _persistent_epoch(self, acts, labels, step_rows=None) -> bool:
        """One client epoch on the adopted persistent executor, made un-killable: the shard's
        weights / optimizer state / counters are copied first (`TailEngine.snapshot_state`);
        if the launch's in-launch waits gave up on ANY Bob rank (a hand-off timeout, the peer-
        mapped fc2 exchange across xGMI failing, an injected fault), every Bob rank restores
        its copy, the peer-mapped region is re-armed collectively, and the job continues on the
        launch-per-stage executor from this epoch on (reported as `server_executor_fallback`).
        Returns False when the caller must run this epoch on launch-per-stage.  Collective over
        the Bob ranks (one small all-reduce per client epoch when tensor-parallel).

        Fault injection (tests): SL_FAULT_PERSIST_EPOCH="TP_RANK:EPOCH:STEP" stops every
        workgroup of TP rank TP_RANK's launch at step STEP of its EPOCH-th persistent epoch
        (0-based), as an in-launch failure would."""
        from ..engine import resident
        if not hasattr(self, "_failsafe"):
            self._failsafe = resident.Failsafe(self.tail, self.bob_slot, self.B, group=self.comm.tp_group,
                                               enabled=getattr(self.args, "persistent_failsafe", "on") != "off")
        fs = self._failsafe
        if fs.run(self.server_executor, acts, labels, step_rows):
            return True
        self.server_executor = "launch_per_stage"
        st = getattr(self, "resident_status", None) or {}
        st["fallback"] = fs.fallback
        self.resident_status = st
        return False

    def server_epoch(self, acts, labels):
        """One pass of Bob's optimizer over one client's cached activations (batch order as
        cached).  Full batches run as HIP-graph chunks of GRAPH_STEPS steps when possible."""
        n, B = labels.numel(), self.B
        if acts.dtype != torch.float32:          # --act_dtype bf16: the kernels compute in fp32
            acts = acts.float()
        s = 0
        G = self.GRAPH_STEPS
        la = self.tail.lookahead_ok(B)
        pre = False
        if n >= B and (self._use_resident() or self._use_hybrid()):
            # one persistent launch for every full batch: a narrow (tensor-parallel) shard with
            # its weights and Adam state on-chip (csrc/resident.hip), or a wide shard with fc2 /
            # fc3 on-chip and fc1 streamed (csrc/hybrid.hip); on an in-launch failure the shard
            # is rolled back and this epoch (and every later one) runs launch-per-stage below
            if self._persistent_epoch(acts.contiguous(), labels.contiguous()):
                self.comm.progress()
                return
        if self._use_graphs() and n // B >= G:
            key = (B, G, acts.shape[1])
            gs = getattr(self, "_graphed", {}).get(key)
            if gs is None:
                from ..engine.graphs import GraphedServerSteps
                if not hasattr(self, "_graphed"):
                    self._graphed = {}
                gs = self._graphed[key] = GraphedServerSteps(self.tail, self.bob_slot, B, G, acts.shape[1])
            ng = (n // B // G) * G
            pre = gs.run(acts, labels, ng)
            self.comm.progress()
            s = ng * B
        elif la and n >= B:
            self.tail.lookahead_prologue(acts[:B])
            pre = True
            if getattr(self.args, "native_epoch", True) and self.tail.native_epoch_ok(B):
                # the whole epoch's steps issued from C++ (csrc/engine.cpp), same numerics
                self.tail.run_native_epoch(acts.contiguous(), labels.contiguous(), self.bob_slot, B, pre)
                self.comm.progress()
                return
        for s in range(s, n, B):
            # look ahead only to a full batch (the prologue / slabs are sized for B rows)
            nxt = acts[s + B:s + 2 * B] if la and s + 2 * B <= n else None
            self.server_step(acts[s:s + B], labels[s:s + B], pre=pre, x_next=nxt)
            self.comm.progress()
            pre = nxt is not None

    def train_and_backward(self, unlearn_request_from_alices, unlearn_id):
        """Reference `bob.train_and_backward` (data_entities_vanilla_sisa.py:294-315)."""
        self.bob_log.info("Global Training")
        self.switch_mode_to_train()
        samples = 0
        self.prefetch_activations(unlearn_request_from_alices, unlearn_id)
        plan = None
        for _ in _progress(range(self.args.server_epochs), self.show, desc="Epochs", ascii=" >="):
            caches = []
            for cid in range(1, self.k + 1):
                if cid in unlearn_request_from_alices:
                    caches.append(self.get_activation_and_labels(cid, unlearned=True, unlearn_id=unlearn_id))
                else:
                    caches.append(self.get_activation_and_labels(cid, unlearned=False))
            if not self.is_bob:
                continue
            n_all = sum(int(c[1].numel()) for c in caches)
            if (self._use_resident() or self._use_hybrid()) and n_all > 0:
                # the whole server epoch, every client's batches in order (short final batches
                # included), as ONE persistent-executor call: one launch (or a few, past the 2 GB
                # input offsets) instead of one per client plus a launch-per-stage tail batch each.
                # The plan (a padded copy for several clients) is rebuilt whenever a cache tensor
                # is not the one it was built from (storage, shape or in-place version changed),
                # and lives only for this call
                key = tuple((a.data_ptr(), tuple(a.shape), a._version, y.data_ptr(), y.numel(), y._version)
                            for a, y in caches)
                if plan is None or plan[0] != key:
                    cs = [(a if a.dtype == torch.float32 else a.float(), y) for a, y in caches]
                    plan = (key, self.tail.padded_plan(cs, self.B))
                X, Y, rows = plan[1]
                with self.tracer.gpu_span("server_epoch[all]", samples=n_all):
                    ok = self._persistent_epoch(X.contiguous(), Y.contiguous(), rows)
                self.comm.progress()
                if ok:
                    samples += n_all
                    continue
            for cid, (acts, labels) in enumerate(caches, 1):
                with self.tracer.gpu_span(f"server_epoch[alice{cid}]", samples=int(labels.numel())):
                    self.server_epoch(acts, labels)
                samples += labels.numel()
        self.bob_log.info("Global training completed.")
        self.comm.barrier()
        return samples

    def inference(self, x):
        return self.tail.forward(x)


class ControlSession(SisaSession):
    """`--control`: SISA semantics with Alice_1 trained on filtered data from the start."""
    mode = "control"
