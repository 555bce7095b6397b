"""SISA with concatenated client embeddings (`--sisa --concat`).

Reference: `/root/reference/data_entities_sisa_concat.py` + `models.py:66-82`
(`model2_sisa_concat(k)`: fc1 takes 5408*k inputs, fc3 emits 100*k logits).
The reference concatenates along the *batch* dimension, then iterates single
samples and crashes in `torch.flatten(x, 1)` (Q3); its eval is a TODO.  The
layer shapes only make sense for a **feature** concatenation, so this module
pins the semantics SURVEY H6 recommends (documented in docs/DEVIATIONS.md):

* server step t takes batch t of every Alice's cached activations and lays them
  side by side: row b = [act_1[b] | act_2[b] | ... | act_k[b]] (zeros for an Alice
  whose cache is exhausted or whose last batch is shorter);
* logits are k heads of 100: loss = sum_j CE(logits[:, 100j:100j+100], y_j), each
  a mean over Alice j's valid rows (rows without a sample carry ignore_index);
* eval feeds Alice j's activation in slot j and zeros elsewhere and reads head j;
* with `--concat_unlearn` the SISA unlearn/retrain tail is appended (BASELINE
  config 5; the reference concat schedule has no unlearning step).

The activation caches are replicated on every Bob TP rank by the dump (p2p
multicast = the all-gather of client embeddings), so the per-step concat is a
device-local gather into one [B, 5408k] buffer.
"""
from __future__ import annotations

import torch

from ..config import CUT_FEATURES
from ..models import ServerTailSisaConcat, sisa_server_spec
from .base import _progress
from .sisa import SisaSession


class ConcatSession(SisaSession):
    mode = "concat"

    def _decide_resident(self) -> bool:
        # k cross-entropy groups (SISA-concat's heads): the resident executor serves one
        return False

    def bob_module_and_spec(self):
        return (self.make_bob_module(ServerTailSisaConcat, self.k),
                sisa_server_spec(self.k, concat=True))

    def _build_bob(self):
        super()._build_bob()
        self.tail.ce_groups = self.k         # one 100-way cross-entropy head per client

    def cut_width_in(self) -> int:
        return CUT_FEATURES

    def bob_out_width(self) -> int:
        return 100

    def bob_infer(self, act, cid):
        """Eval: Alice_cid's activation in slot cid, zeros elsewhere; returns head cid.  Only
        fc1's column block of slot cid and fc3's head-cid rows are multiplied
        (`TailEngine.forward_block`): the zero blocks of the padded input add nothing, so this is
        the same function at 1/k of fc1's work."""
        j = cid - 1
        return self.tail.forward_block(act, j * CUT_FEATURES, 100 * j, 100)

    def concat_step(self, caches, t: int):
        k, B = self.k, self.B
        rows = []
        for acts, labels in caches:
            rows.append(max(0, min(B, labels.numel() - t * B)))
        M = max(rows)
        X = torch.zeros(M, CUT_FEATURES * k, device=self.device)
        Y = torch.full((M, k), -100, dtype=torch.int64, device=self.device)
        scale = torch.zeros(M, k, device=self.device)
        for j, ((acts, labels), r) in enumerate(zip(caches, rows)):
            if r == 0:
                continue
            X[:r, j * CUT_FEATURES:(j + 1) * CUT_FEATURES] = acts[t * B:t * B + r]
            Y[:r, j] = labels[t * B:t * B + r]
            scale[:r, j] = 1.0 / r
        out = self.tail.forward(X, train=True)                       # [M, 100k]
        _, d = self.ops.softmax_ce(out.view(M * k, 100), Y.view(-1), 1.0)
        d = (d.view(M, k, 100) * scale.view(M, k, 1)).view(M, 100 * k)
        self.tail.backward_dgrad(d, need_dx=False)
        self.tail.backward_step(self.bob_slot)
        return sum(rows)

    def concat_epoch(self, caches) -> int:
        """One server epoch = `concat_step(caches, t)` for every t, restructured for the GPU:
        the concatenated inputs, head labels and per-head CE scales of the whole epoch are
        laid out once ([T*B, 5408k] etc.), and the steps are pipelined like the SISA server
        epoch: each step's grouped wgrad + optimizer launch also forms the next step's fc1
        product with the updated weights (`TailEngine.group_step(x_next=...)`), so fc1 —
        5408k inputs wide — is read once per step instead of twice.  Same math per step."""
        k, B, dev = self.k, self.B, self.device
        ns = [c[1].numel() for c in caches]
        T = max(-(-n // B) for n in ns) if ns else 0
        if T == 0:
            return 0
        X = torch.zeros(T * B, CUT_FEATURES * k, device=dev)
        Y = torch.full((T * B, k), -100, dtype=torch.int64, device=dev)
        scale = torch.zeros(T * B, k, device=dev)
        rows = [[max(0, min(B, n - t * B)) for n in ns] for t in range(T)]
        for j, ((acts, labels), n) in enumerate(zip(caches, ns)):
            X[:n, j * CUT_FEATURES:(j + 1) * CUT_FEATURES] = acts
            Y[:n, j] = labels
            r = torch.tensor([rows[t][j] for t in range(T)], dtype=torch.float32)
            sc = torch.where(r > 0, 1.0 / r.clamp(min=1), torch.zeros_like(r)).repeat_interleave(B)
            scale[:, j] = sc.to(dev) * (Y[:, j] != -100)
        Ms = [max(r) for r in rows]
        tail = self.tail
        if tail.native_epoch_ok(B):
            # the fused server step on the concatenated rows (the grouped cross-entropy head):
            # every step takes B rows; rows past a step's M_t are zero with every label
            # ignored, so they add nothing to any gradient — the same step as on M_t rows.
            # Issued from C++ (csrc/engine.cpp), or step by step from here with the same
            # launches (`--python_epoch`; bitwise equal, tests/test_split_native_gpu.py)
            tail.lookahead_prologue(X[:B])
            if getattr(self.args, "native_epoch", True):
                tail.run_native_epoch(X, Y, self.bob_slot, B, True, gscale=scale)
            else:
                for t in range(T):
                    sl = slice(t * B, (t + 1) * B)
                    tail.train_fwd_bwd3(X[sl], Y[sl].reshape(-1), need_dx=False, pre=True, gscale=scale[sl])
                    tail.fused_step(self.bob_slot, x_next=X[(t + 1) * B:(t + 2) * B] if t + 1 < T else None)
                    self.comm.progress()
            self.comm.progress()
            return sum(sum(r) for r in rows)
        grouped = tail.grouped_ok()
        pre = False
        for t in range(T):
            M = Ms[t]
            x = X[t * B:t * B + M]
            out = tail.forward(x, train=True, pre=pre)                    # [M, 100k]
            _, d = self.ops.softmax_ce(out.view(M * k, 100), Y[t * B:t * B + M].reshape(-1), 1.0)
            d = (d.view(M, k, 100) * scale[t * B:t * B + M].view(M, k, 1)).view(M, 100 * k)
            tail.backward_dgrad(d, need_dx=False)
            pre = False
            if grouped:
                nxt = X[(t + 1) * B:(t + 1) * B + Ms[t + 1]] if t + 1 < T else None
                x_next = nxt if (nxt is not None and tail.grouped_ok(nxt.shape[0])) else None
                tail.group_step(self.bob_slot, x_next=x_next)
                pre = x_next is not None
            else:
                tail.backward_step(self.bob_slot)
            self.comm.progress()
        return sum(sum(r) for r in rows)

    def train_and_backward(self, unlearn_request_from_alices, unlearn_id):
        self.bob_log.info("Global Training")
        self.switch_mode_to_train()
        samples = 0
        self.prefetch_activations(unlearn_request_from_alices, unlearn_id)
        for _ in _progress(range(self.args.server_epochs), self.show, desc="Epochs", ascii=" >="):
            caches = []
            for cid in range(1, self.k + 1):
                if cid in unlearn_request_from_alices:
                    caches.append(self.get_activation_and_labels(cid, unlearned=True, unlearn_id=unlearn_id))
                else:
                    caches.append(self.get_activation_and_labels(cid, unlearned=False))
            if self.is_bob:
                samples += self.concat_epoch(caches)
        self.bob_log.info("Global training completed.")
        self.comm.barrier()
        return samples
