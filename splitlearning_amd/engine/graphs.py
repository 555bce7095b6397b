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
Numerics are identical to the eager path (same step counts, same seeds).

Requires a single-GPU tail (TP degree 1): a tensor-parallel step contains a
collective and runs eagerly.
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
        self.x = torch.zeros(G * B, k_in, device=dev)
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
        for key, n in (("dgrad", kmax), ("fwd", nmax), ("fc2p", nmax), ("dz1p", kmax)):
            ops._workspace(dev, 16 * B * n, key)
        torch.cuda.synchronize(dev)
        fwd0 = tail.fwd_count
        self.graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(self.graph, stream=s):
                fused = tail.fused3_ok()
                for i in range(G):
                    xs = self.x[i * B:(i + 1) * B]
                    ys = self.y[i * B:(i + 1) * B]
                    dseeds = [self.seed_tab[i, l] for l in range(self.L)]
                    if fused:
                        tail.train_fwd_bwd3(xs, ys, need_dx=False, dseeds=dseeds)
                        tail.fused_step(slot, t=1, dyn=self.opt_tab[i])
                    else:
                        out = tail.forward(xs, train=True, dseeds=dseeds)
                        _, d = ops.softmax_ce(out, ys, 1.0 / B)
                        tail.backward_dgrad(d, need_dx=False)
                        tail.backward_step(slot, t=1, dyn=self.opt_tab[i])
        torch.cuda.current_stream(dev).wait_stream(s)
        tail.fwd_count = fwd0           # capture does not execute: restore the host counters
        self._tabs = None

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

    def run(self, acts: torch.Tensor, labels: torch.Tensor, nsteps: int):
        """Run the first `nsteps` (a multiple of G) full batches of (acts, labels)."""
        G, B = self.G, self.B
        assert nsteps % G == 0 and nsteps * B <= labels.numel()
        opt_all, seed_all = self._epoch_tables(nsteps)
        for c in range(nsteps // G):
            r0 = c * G * B
            self.x.copy_(acts[r0:r0 + G * B])
            self.y.copy_(labels[r0:r0 + G * B])
            self.opt_tab.copy_(opt_all[c * G:(c + 1) * G])
            self.seed_tab.copy_(seed_all[c * G:(c + 1) * G])
            self.graph.replay()
        self.slot.t += nsteps
        self.tail.fwd_count += nsteps
