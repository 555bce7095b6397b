"""HIP-graph execution of Bob's SISA server epoch.

Bob's server phase (data_entities_vanilla_sisa.py:298-313) is a long run of
identical-shape steps — forward, CE, dgrads, fused wgrad+Adam — over the cached
activations.  Eagerly, each step costs ~11 kernel launches from Python; a graph of
G consecutive steps replays all of them with one host call and no inter-launch gaps.

What varies between replays is handled without re-capture:
* the batch: the chunk's G*B cached rows are copied (device-to-device) into a
  static staging buffer the graph reads;
* Adam's bias corrections {lr/(1-b1^t), 1/sqrt(1-b2^t)} and the per-layer dropout
  seeds: kernels read them from small static device tables (`SlOpt.dyn`,
  `Epi.dseed`), refreshed per chunk by a device-to-device copy from per-epoch tables
  that the host fills once.
* the fc1 look-ahead (TailEngine.fused_step(x_next=...)): step i of the graph
  pre-computes fc1's product for step i+1; the staging buffer holds G+1 batches so
  the last step pre-computes the first batch of the next chunk, and `run` starts the
  chain with an eager `lookahead_prologue`.
Numerics are identical to the eager `SisaSession.server_epoch` loop (same step counts,
seeds and kernel sequence).

A tensor-parallel tail is captured too when its all-reduce is the native
(capturable) RCCL communicator (parallel/rccl.py).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.rng import step_seed
from .slots import OptSlot
from .tail import TailEngine


class GraphedServerSteps:
    def __init__(self, tail: TailEngine, slot: OptSlot, B: int, G: int, k_in: int):
        if tail.tp_size != 1 and not getattr(tail.allreduce, "capturable", False):
            raise ValueError("graph capture of a tensor-parallel tail needs the native RCCL all-reduce")
        if slot.cfg.kind != "adam":
            raise ValueError("graphed server steps implement the SISA Adam slot")
        self.tail, self.slot, self.B, self.G = tail, slot, B, G
        dev = tail.device
        self.L = len(tail.layers)
        self.x = torch.zeros((G + 1) * B, k_in, device=dev)
        self.y = torch.zeros(G * B, dtype=torch.int64, device=dev)
        self.opt_tab = torch.zeros(G, 2, device=dev)
        self.seed_tab = torch.zeros(G, self.L, 2, dtype=torch.int32, device=dev)
        for L in tail.layers:      # optimizer state must exist (and stay put) before capture
            slot.state(f"{L.spec.name}.weight", L.W)
            slot.state(f"{L.spec.name}.bias", L.b)
        ops = tail.ops
        # scratch slabs must be allocated outside the capture (they are shared with eager calls)
        kmax = max(max(L.W.shape[1] for L in tail.layers), k_in)
        nmax = max(L.W.shape[0] for L in tail.layers)
        for key, n in (("dgrad", kmax), ("fwd", nmax), ("fc2p", nmax), ("dz1p", kmax), ("head", nmax)):
            ops._workspace(dev, 16 * B * n, key)
        # the look-ahead slab buffer the graph reads: kept here and written by run()'s
        # prologue directly, so a later growth of the shared workspace cannot leave the
        # graph reading a buffer nobody writes any more
        self.pn = tail.lookahead_slabs(B) if tail.lookahead_ok(B) else None
        self._ws = [ops._workspace(dev, 16 * B * n, key) for key, n in
                    (("dgrad", kmax), ("fwd", nmax), ("fc2p", nmax), ("dz1p", kmax), ("head", nmax))]
        torch.cuda.synchronize(dev)
        fwd0 = tail.fwd_count
        self.graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(self.graph, stream=s):
                fused = tail.fused3_ok()
                self.lookahead = fused and tail.lookahead_ok(B)
                if self.lookahead:
                    tail._pre = self.pn                     # filled by run()'s prologue
                for i in range(G):
                    xs = self.x[i * B:(i + 1) * B]
                    ys = self.y[i * B:(i + 1) * B]
                    dseeds = [self.seed_tab[i, l] for l in range(self.L)]
                    if fused:
                        tail.train_fwd_bwd3(xs, ys, need_dx=False, dseeds=dseeds, pre=self.lookahead)
                        xn = self.x[(i + 1) * B:(i + 2) * B] if self.lookahead else None
                        tail.fused_step(slot, t=1, dyn=self.opt_tab[i], x_next=xn)
                    else:
                        out = tail.forward(xs, train=True, dseeds=dseeds)
                        _, d = ops.softmax_ce(out, ys, 1.0 / B)
                        tail.backward_dgrad(d, need_dx=False)
                        tail.backward_step(slot, t=1, dyn=self.opt_tab[i])
        torch.cuda.current_stream(dev).wait_stream(s)
        tail.fwd_count = fwd0           # capture does not execute: restore the host counters
        tail._pre = None

    def _epoch_tables(self, nsteps: int):
        """Per-step Adam scalars and dropout seeds for the next `nsteps` steps."""
        cfg = self.slot.cfg
        t = np.arange(self.slot.t + 1, self.slot.t + nsteps + 1, dtype=np.float64)
        opt = np.stack([cfg.lr / (1.0 - cfg.beta1 ** t), 1.0 / np.sqrt(1.0 - cfg.beta2 ** t)], 1)
        seeds = np.zeros((nsteps, self.L, 2), dtype=np.uint32)
        for i in range(nsteps):
            for l in range(self.L):
                s = step_seed(self.tail.seed_base, l, self.tail.fwd_count + i + 1)
                seeds[i, l, 0] = s & 0xFFFFFFFF
                seeds[i, l, 1] = s >> 32
        dev = self.tail.device
        return (torch.from_numpy(opt.astype(np.float32)).to(dev),
                torch.from_numpy(seeds.view(np.int32)).to(dev))

    def run(self, acts: torch.Tensor, labels: torch.Tensor, nsteps: int) -> bool:
        """Run the first `nsteps` (a multiple of G) full batches of (acts, labels).
        Returns True when the look-ahead for the following full batch (rows
        nsteps*B ... +B) is pending in the tail (pass `pre=True` to its step)."""
        G, B = self.G, self.B
        n = labels.numel()
        assert nsteps % G == 0 and nsteps * B <= n
        opt_all, seed_all = self._epoch_tables(nsteps)
        if self.lookahead:
            self.tail.lookahead_prologue(acts[:B], out=self.pn)
        for c in range(nsteps // G):
            r0 = c * G * B
            r1 = min(n, r0 + (G + 1) * B)
            self.x[:r1 - r0].copy_(acts[r0:r1])
            self.y.copy_(labels[r0:r0 + G * B])
            self.opt_tab.copy_(opt_all[c * G:(c + 1) * G])
            self.seed_tab.copy_(seed_all[c * G:(c + 1) * G])
            self.graph.replay()
        self.slot.t += nsteps
        self.tail.fwd_count += nsteps
        pending = self.lookahead and nsteps * B + B <= n
        self.tail._pre = self.pn if pending else None
        return pending
