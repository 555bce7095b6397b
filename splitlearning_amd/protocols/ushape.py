"""U-shape split learning (default mode): Alice conv front -> Bob MLP middle ->
Alice head + loss.  Labels never leave the client.

Reference: `/root/reference/data_entities.py` (alice `:23-128`, bob `:131-180`),
schedule `split_nn.py:47-60`.  Per batch (data_entities.py:65-81) the reference
does an `inference` RPC forward and a dist-autograd backward that crosses the
process boundary twice, then a DistributedOptimizer Adam step over
model3 + Bob + model1.  Here: activation Alice->Bob, Bob's [B,100] output
Bob->Alice, head forward/CE/backward on Alice, dL/d(Bob output) Alice->Bob,
Bob dgrad -> cut gradient Bob->Alice (posted async, overlapping Bob's fused
wgrad+Adam), Alice's fused conv backward+Adam.  Bob keeps one Adam slot per
Alice (Q8).  The reference crashes after training because the U-shape bob has
no `eval_request_breakdown` (Q1); this module implements it and the U-shape
unlearn request so the reference schedule runs to completion.
"""
from __future__ import annotations

import torch

from ..config import CUT_FEATURES
from ..engine.slots import OptSlot, adam
from ..engine.tail import TailEngine
from ..models import ClientFront, Head, ServerTailUShape, head_spec, ushape_server_spec
from .base import AliceState, Session, _progress
from .split_native import (native_remote_role, native_split_ok, persistent_ushape_ok, run_native_remote_epoch,
                           run_native_split_epoch, run_persistent_ushape_epoch)


class UShapeSession(Session):
    mode = "ushape"

    def front_module(self):
        return ClientFront()

    def alice_optim(self):
        return adam(self.args.lr)

    def bob_optim(self):
        return adam(self.args.lr)

    def bob_module_and_spec(self):
        return self.make_bob_module(ServerTailUShape), ushape_server_spec()

    def _extend_alice(self, a: AliceState):
        torch.manual_seed(self.seed + 2000 + a.cid)
        a.head = TailEngine(Head(), head_spec(), self.device)

    def bob_slot(self, cid: int) -> OptSlot:
        s = self.bob_slots.get(cid)
        if s is None:
            s = self.bob_slots[cid] = OptSlot(self.bob_optim())
        return s

    # ------------------------------------------------------------------ weights (model1 + model3)
    def give_weights(self, cid: int):
        a = self.alices[cid]
        return [{k: v.detach().clone() for k, v in a.front.module.state_dict().items()},
                {k: v.detach().clone() for k, v in a.head.module.state_dict().items()}]

    def _flat_client_weights(self, a):
        return torch.cat([a.front.flat_weights(), a.head.flat_weights()])

    def _load_flat_client_weights(self, a, flat):
        n = a.front.flat_numel
        a.front.load_flat_weights(flat[:n])
        a.head.load_flat_weights(flat[n:])

    def _client_flat_numel(self) -> int:
        return 32 * 9 + 32 + 100 * 10 + 10

    def _client_state(self, a):
        return {"model1": {k: v.detach().cpu() for k, v in a.front.module.state_dict().items()},
                "model3": {k: v.detach().cpu() for k, v in a.head.module.state_dict().items()}}

    def _load_client_state(self, a, sd):
        a.front.module.load_state_dict({k: v.to(self.device) for k, v in sd["model1"].items()})
        a.head.load_full_state_dict(sd["model3"])

    def reset_model(self, cid: int):
        a = self.alices[cid]
        a.front.reset_parameters(self.args.true_reset)
        with torch.no_grad():
            a.head.reset_parameters()

    # ------------------------------------------------------------------ one U-shape step
    def head_fused(self, M: int) -> bool:
        """Whether Alice's head runs as one `_C.head_step` launch for a batch of M.  Every
        rank evaluates this same rule (device kernels + the fixed 100 -> 10 head), so Bob
        knows that the dL/d(mid) he receives already carries his final ReLU's backward."""
        return hasattr(self.ops, "head_step_") and M * 100 <= 4096 and M * 10 <= 1024

    def head_train(self, a, mid, labels, t: int):
        """Alice's head on Bob's output: forward, CE, dL/d(mid) and the head's optimizer step
        (data_entities.py:74-81).  One launch when the head fits `_C.head_step`; that launch
        also applies the [mid > 0] mask of Bob's final ReLU (mid is that ReLU's output)."""
        if self.head_fused(mid.shape[0]):
            assert a.head.head_step_ok(mid.shape[0])
            _, dmid = a.head.head_step(mid, labels, a.slot, t, prefix="head.", mask_input=True)
            return dmid
        logits = a.head.forward(mid, train=True)
        _, dlog = self.ops.softmax_ce(logits, labels, 1.0 / mid.shape[0])
        dmid = a.head.backward_dgrad(dlog, need_dx=True)
        a.head.backward_step(a.slot, t, prefix="head.")
        return dmid

    def split_step(self, cid: int, idx, B: int):
        host = self.host(cid)
        a = self.alices.get(cid)
        act = am = labels = None
        if a is not None:
            act, am, labels = a.front.forward(a.train, idx, with_labels=True)
        act_b = self.act_to_bob(cid, act, B)
        out = self.tail.forward(act_b, train=True) if self.is_bob else None
        mid = self.from_bob(cid, out, (B, 100))
        dmid = None
        t = None
        if a is not None:
            t = a.slot.tick()
            dmid = self.head_train(a, mid, labels, t)
        dmid_b = self.to_bob(cid, dmid, (B, 100))
        dxp = self.tail.backward_dgrad(dmid_b, need_dx=True, premasked=self.head_fused(B)) if self.is_bob else None
        fin = self.comm.reduce_to_async(dxp, host, self.bob_ranks, (B, CUT_FEATURES), torch.float32)
        if self.is_bob:
            self.tail.backward_step(self.bob_slot(cid))
        dx = fin()
        if a is not None:
            a.front.backward_step(dx, act, am, a.train, idx, a.slot, t=t, prefix="front.")

    def split_epoch(self, cid: int, order, n: int):
        """U-shape training of Alice_cid over `order` (n samples), pipelined like
        VanillaSession.split_epoch: per batch i, Bob's forward, the head + CE + head step on
        Alice, Bob's data gradients, Alice's conv backward + step and her forward of batch
        i+1 (sent to Bob) — and only then Bob's wgrad + Adam of both layers in one launch,
        which also forms batch i+1's fc1 product with the updated weights (no separate fc1
        forward read).  Same per-batch math and update order as `split_step`.  When no Bob
        shard shares the Alice's GPU (`split_lookahead`), Bob's update is issued right after
        the cut gradient leaves instead, so it runs during her backward and next forward."""
        B = self.B
        a = self.alices.get(cid)
        host = self.host(cid)
        spans = [(s, min(s + B, n)) for s in range(0, n, B)]
        if not spans:
            return
        if order is not None and persistent_ushape_ok(self, cid) and run_persistent_ushape_epoch(self, cid, order):
            return                                # the whole epoch in one launch, state on-chip
        if order is not None and native_split_ok(self, cid, "ushape"):
            run_native_split_epoch(self, cid, order, "ushape")   # the same launches, issued from C++
            return
        role = native_remote_role(self, cid, "ushape")   # collective over the Alice's and Bob's ranks
        if role is not None:                      # remote Alice: each side's half from C++
            run_native_remote_epoch(self, cid, order, n, "ushape", role)
            return
        grouped = self.is_bob and self.tail.grouped_ok()
        la = self.split_lookahead(cid)

        def alice_fwd(span):
            s, e = span
            idx = order[s:e] if order is not None else None
            act = am = labels = None
            if a is not None:
                act, am, labels = a.front.forward(a.train, idx, with_labels=True)
            return idx, act, am, labels, self.act_to_bob(cid, act, e - s)

        cur = alice_fwd(spans[0])
        pre = False
        for i, (s, e) in enumerate(spans):
            idx, act, am, labels, act_b = cur
            M = e - s
            out = self.tail.forward(act_b, train=True, pre=pre) if self.is_bob else None
            mid = self.from_bob(cid, out, (M, 100))
            dmid = t = None
            if a is not None:
                t = a.slot.tick()
                dmid = self.head_train(a, mid, labels, t)
            dmid_b = self.to_bob(cid, dmid, (M, 100))
            dxp = (self.tail.backward_dgrad(dmid_b, need_dx=True, premasked=self.head_fused(M))
                   if self.is_bob else None)
            dx = self.comm.reduce_to(dxp, host, self.bob_ranks, (M, CUT_FEATURES), torch.float32)
            pre = False
            if self.is_bob and not la:           # Alice remote from every Bob shard: the
                if grouped:                      # update overlaps her backward + next forward
                    self.tail.group_step(self.bob_slot(cid), x_next=None)
                else:
                    self.tail.backward_step(self.bob_slot(cid))
            if a is not None:
                a.front.backward_step(dx, act, am, a.train, idx, a.slot, t=t, prefix="front.", defer=True)
            nxt = alice_fwd(spans[i + 1]) if i + 1 < len(spans) else None
            if self.is_bob and la:
                if grouped:
                    x_next = nxt[4] if (la and nxt is not None and self.tail.grouped_ok(nxt[4].shape[0])) else None
                    self.tail.group_step(self.bob_slot(cid), x_next=x_next)
                    pre = x_next is not None
                else:
                    self.tail.backward_step(self.bob_slot(cid))
            cur = nxt
        if a is not None:
            a.front.flush()          # the last step's deferred client update

    def _run_epochs(self, cid: int, order_fn, n: int):
        for _ in _progress(range(self.args.epochs), self.show, desc="Epochs", ascii=" >="):
            a = self.alices.get(cid)
            order = order_fn(a) if a is not None else None
            self.split_epoch(cid, order, n)

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
        self._run_epochs(client_id, lambda al: al.train.shuffled_order(al.gen), self.n_train[client_id])
        self.last_alice_id = client_id

    def unlearn_request(self, client_id: int, omit_label: int):
        """U-shape unlearning (absent in the reference, Q1): reset + fresh Adam states
        (client and Bob-side slot) + retrain on the filtered shard."""
        self.bob_log.info(f"Unlearn Request for Alice-{client_id}")
        a = self.alices.get(client_id)
        order = None
        if a is not None:
            a.logger.info("Retraining")
            self.reset_model(client_id)
            a.slot = OptSlot(self.alice_optim())
            order = self.filtered_order(a, omit_label)
            a.unlearn_order = order
            a.logger.info("Retraining dataset: {}".format(self.label_counter(a, order)))
            a.logger.info("Test dataset (retraining): {}".format(a.test.label_counter()))
        self.bob_slots[client_id] = OptSlot(self.bob_optim())
        n = torch.tensor([order.numel() if order is not None else 0], dtype=torch.int64, device=self.device)
        n = int(self.comm.multicast(n if a is not None else None, self.host(client_id),
                                    range(self.comm.world), (1,), torch.int64).item())
        self._run_epochs(client_id, lambda al: al.unlearn_order, n)

    # ------------------------------------------------------------------ eval hooks
    def bob_out_width(self) -> int:
        return 100

    def client_logits(self, cid: int, bob_out):
        return self.alices[cid].head.forward(bob_out, train=False)

    def inference(self, x):
        return self.tail.forward(x)
