"""Vanilla split learning (`--vanilla`): Alice conv front -> Bob MLP tail + loss
(labels go to Bob), round-robin clients with peer-to-peer weight relay, SGD with
momentum, and the "unlearn = retrain Alice_1 without the omitted label" loop.

Reference: `/root/reference/data_entities_vanilla.py` (alice `:24-207`, bob
`:210-301`), schedule `split_nn.py:47-60`.  Per batch the reference makes ~4 RPC
round trips (activation+labels, dist-autograd gradient, remote optimizer step,
context cleanup).  Here a batch is: one packed p2p message
Alice->Bob (activation + labels), Bob forward/CE/dgrad, the cut gradient
Bob->Alice posted asynchronously, Bob's fused wgrad+SGD kernels overlapping that
transfer, then Alice's fused conv backward+SGD.  Bob keeps one momentum slot per
Alice (the reference's per-Alice DistributedOptimizer, Q8), re-created on unlearn.
"""
from __future__ import annotations

import torch

from ..config import CUT_FEATURES
from ..engine.slots import OptSlot, sgd_momentum
from ..models import ServerTailSisa, sisa_server_spec
from .base import Session, _progress
from .split_native import (native_remote_role, native_split_ok, persistent_vanilla_ok, run_native_remote_epoch,
                           run_native_split_epoch, run_persistent_vanilla_epoch)


class VanillaSession(Session):
    mode = "vanilla"

    def alice_optim(self):
        return sgd_momentum(self.args.lr)

    def bob_optim(self):
        return sgd_momentum(self.args.lr)

    def bob_module_and_spec(self):
        return self.make_bob_module(ServerTailSisa), sisa_server_spec()

    def bob_slot(self, cid: int) -> OptSlot:
        s = self.bob_slots.get(cid)
        if s is None:
            s = self.bob_slots[cid] = OptSlot(self.bob_optim())
        return s

    def before_eval(self):
        # Q7: the vanilla Bob never switches to eval mode -> dropout stays on during evaluation
        if self.args.eval_dropout_fix:
            self.switch_mode_to_eval()

    # ------------------------------------------------------------------ one split step
    def split_step(self, cid: int, idx, B: int):
        """One batch of split training for Alice_cid (collective over host + Bob ranks)."""
        host = self.host(cid)
        a = self.alices.get(cid)
        act = am = labels = None
        if a is not None:
            act, am, labels = a.front.forward(a.train, idx, with_labels=True)
        act_b, lab_b = self.send_act_labels(cid, act, labels, B)
        dxp = None
        fused = self.is_bob and self.tail.fused3_ok()
        if self.is_bob:
            if fused:
                _, dxp = self.tail.train_fwd_bwd3(act_b, lab_b, need_dx=True)
            else:
                out = self.tail.forward(act_b, train=True)
                _, dout = self.ops.softmax_ce(out, lab_b, 1.0 / B)
                dxp = self.tail.backward_dgrad(dout, need_dx=True)
        fin = self.comm.reduce_to_async(dxp, host, self.bob_ranks, (B, CUT_FEATURES), torch.float32)
        if self.is_bob:
            if fused:
                self.tail.fused_step(self.bob_slot(cid))
            else:
                self.tail.backward_step(self.bob_slot(cid))
        dx = fin()
        if a is not None:
            a.front.backward_step(dx, act, am, a.train, idx, a.slot)

    def split_epoch(self, cid: int, order, n: int):
        """Split training of Alice_cid over `order` (n samples), pipelined so Bob never
        re-reads fc1 for a forward: per batch i, Bob's forward + CE + data gradients, the
        cut gradient to Alice, Alice's backward + step, Alice's forward of batch i+1 (sent
        to Bob), and only then Bob's wgrad + optimizer, whose kernel also forms batch i+1's
        fc1 product with the freshly updated weights (look-ahead, TailEngine.fused_step).
        Same math and update order as `split_step` per batch (both sides step on batch i
        before either runs batch i+1); on one GPU the reordering is free because the
        launches were serial anyway.  When no Bob shard shares the Alice's GPU
        (`split_lookahead`), Bob's update is issued right after the cut gradient leaves
        instead, so it runs during her backward and next forward (§3.2 overlap)."""
        B = self.B
        a = self.alices.get(cid)
        host = self.host(cid)
        spans = [(s, min(s + B, n)) for s in range(0, n, B)]
        if not spans:
            return
        if order is not None and persistent_vanilla_ok(self, cid) and run_persistent_vanilla_epoch(self, cid, order):
            return                                # the whole epoch in one launch (csrc/vanilla.hip)
        if order is not None and native_split_ok(self, cid, "vanilla"):
            run_native_split_epoch(self, cid, order, "vanilla")   # the same launches, issued from C++
            return
        role = native_remote_role(self, cid, "vanilla")   # collective over the Alice's and Bob's ranks
        if role is not None:                      # remote Alice: each side's half from C++
            run_native_remote_epoch(self, cid, order, n, "vanilla", role)
            return
        ahead = self.split_lookahead(cid)        # False: Alice remote from every Bob shard
        la = self.is_bob and self.tail.fused3_ok() and self.tail.lookahead_ok(B) and ahead

        def bob_update(x_next):
            if self.tail.fused3_ok():
                self.tail.fused_step(self.bob_slot(cid), x_next=x_next)
                return x_next is not None
            self.tail.backward_step(self.bob_slot(cid))
            return False

        def alice_fwd(span):
            s, e = span
            idx = order[s:e] if order is not None else None
            act = am = labels = None
            if a is not None:
                act, am, labels = a.front.forward(a.train, idx, with_labels=True)
            act_b, lab_b = self.send_act_labels(cid, act, labels, e - s)
            return idx, act, am, act_b, lab_b

        cur = alice_fwd(spans[0])
        pre = False
        for i, (s, e) in enumerate(spans):
            idx, act, am, act_b, lab_b = cur
            M = e - s
            dxp = None
            fused = self.is_bob and self.tail.fused3_ok()
            if self.is_bob:
                if fused:
                    _, dxp = self.tail.train_fwd_bwd3(act_b, lab_b, need_dx=True, pre=pre)
                else:
                    out = self.tail.forward(act_b, train=True)
                    _, dout = self.ops.softmax_ce(out, lab_b, 1.0 / M)
                    dxp = self.tail.backward_dgrad(dout, need_dx=True)
            dx = self.comm.reduce_to(dxp, host, self.bob_ranks, (M, CUT_FEATURES), torch.float32)
            pre = False
            if self.is_bob and not ahead:
                bob_update(None)                  # overlaps the Alice's backward + next forward
            if a is not None:
                a.front.backward_step(dx, act, am, a.train, idx, a.slot, defer=True)
            nxt = alice_fwd(spans[i + 1]) if i + 1 < len(spans) else None
            if self.is_bob and ahead:
                pre = bob_update(nxt[3] if (la and nxt is not None and nxt[3].shape[0] <= 64) else None)
            cur = nxt
        if a is not None:
            a.front.flush()          # the last step's deferred client update

    def _order_len(self, cid, order):
        n = torch.tensor([order.numel() if order is not None else 0], dtype=torch.int64, device=self.device)
        n = self.comm.multicast(n if self.hosts(cid) else None, self.host(cid),
                                [r for r in range(self.comm.world)], (1,), torch.int64)
        return int(n.item())

    # ------------------------------------------------------------------ Bob API
    def train_request(self, client_id: int):
        self.bob_log.info(f"Train Request for Alice-{client_id}")
        a = self.alices.get(client_id)
        if a is not None:
            a.logger.info("Training")
            if self.last_alice_id is None:
                a.logger.info(f"Alice-{client_id} is first client to train")
            else:
                a.logger.info(f"Alice-{client_id} receiving weights from Alice-{self.last_alice_id}")
        if self.last_alice_id is not None:
            self.relay_weights(self.last_alice_id, client_id)
        self._train_over_shuffled(client_id)
        self.last_alice_id = client_id

    def _train_over_shuffled(self, cid):
        for _ in _progress(range(self.args.epochs), self.show, desc="Epochs", ascii=" >="):
            a = self.alices.get(cid)
            order = a.train.shuffled_order(a.gen) if a is not None else None
            self.split_epoch(cid, order, self.n_train[cid])

    def unlearn_request(self, client_id: int, omit_label: int):
        self.bob_log.info(f"Unlearn Request for Alice-{client_id}")
        a = self.alices.get(client_id)
        order = None
        if a is not None:
            a.logger.info("Retraining")
            self.reset_model(client_id)
            a.slot = OptSlot(self.alice_optim())            # new DistributedOptimizer ...
            order = self.filtered_order(a, omit_label)
            a.unlearn_order = order
            a.logger.info("Retraining dataset: {}".format(self.label_counter(a, order)))
            a.logger.info("Test dataset (retraining): {}".format(a.test.label_counter()))
        self.bob_slots[client_id] = OptSlot(self.bob_optim())  # ... with a fresh Bob-side state
        n = self._order_len(client_id, order)
        for _ in _progress(range(self.args.epochs), self.show, desc="Epochs", ascii=" >="):
            self.split_epoch(client_id, order, n)

    def inference(self, x):
        return self.tail.forward(x)

    def train_and_backward(self, x, labels):
        """Bob-local forward + CE + backward + step on one batch (reference
        `bob.train_and_backward`, data_entities_vanilla.py:226-232); returns the loss."""
        out = self.tail.forward(x, train=True)
        loss, dout = self.ops.softmax_ce(out, labels, 1.0 / x.shape[0])
        self.tail.backward_dgrad(dout, need_dx=False)
        self.tail.backward_step(self.bob_slot(0))
        return loss.sum() / x.shape[0]
