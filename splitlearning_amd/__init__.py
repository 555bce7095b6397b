"""splitlearning_amd — MI355X-native split learning + SISA unlearning.

Layers (re-designed MI355X-first):
  runtime/    launcher: process-per-GPU spawn / torchrun entry, data generation
  protocols/  SPMD Bob schedule + per-mode Alice/Bob request semantics
  parallel/   placement of roles on processes, RCCL/gloo p2p + TP collectives
  engine/     fused executors for the client front, server tail, optimizer slots
  ops/        op set: hand-written gfx950 HIP kernels (hip_ops) / eager torch (torch_ops)
  models/     reference-compatible nn.Modules (state_dict layout)
  data/       Dirichlet partition, tensor-only shards, device-resident datasets
  csrc/       HIP/C++ sources of `_C` (built by `python -m splitlearning_amd.build`)
"""
__version__ = "0.1.0"
