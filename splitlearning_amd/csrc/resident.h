// Register-resident server epoch (csrc/resident.hip): one persistent launch runs S Adam/SGD
// steps of Bob's 3-layer tail with every weight, bias and optimizer-state element of a
// narrow shard (a TP = 8 shard of model2_sisa: fc1 625 x 5408, fc2 1000 x 625, fc3 100 x 1000)
// held on-chip (VGPRs and LDS) from the first step to the last.  See resident.hip.
#pragma once
#include "common.h"
#include "ipc_ar.h"

namespace sl {

constexpr int kResThreads = 512;    // one 8-wave workgroup per CU (256 VGPRs per wave)
constexpr int kResTiles = 4;        // fc1 tiles (16 rows x 256 columns) per workgroup
constexpr int kResGroups = 6;       // fc1 column groups (workgroups per 16-row block)
constexpr int kResRows2 = 4;        // fc2 rows (and fc3 columns) per workgroup
constexpr int kResMaxC = 128;       // fc3 width bound (classes)
constexpr int kResSeams = 4;        // A: h1 rows, B: logit partials, C: dlogits, D: dz2 + W2
constexpr int kResShardStride = 32; // counter shards 128 B apart
constexpr int kResMaxRB = 48;       // fc1 row blocks (16 rows; shard width <= 768)
constexpr int kResCounters = kResSeams * 8 + kResMaxRB;   // seam shards, then one per row block

struct ResLayer {
  float *W, *m, *v;       // [N, K] (v unused for SGD)
  float *b, *mb, *vb;     // [N]
};

struct ResArgs {
  ResLayer L1, L2, L3;
  int N1, K1, N2, C;      // shard fc1 rows, fc1 width, fc2 rows, classes
  int N1p, C4;            // N1 rounded up to 4 (hand-off row pitch), C rounded up to 4
  int M, S, G;            // rows per step (<= 16), steps, workgroups
  int nrb, ncb, ngrp;     // fc1 row blocks (16), column blocks (256), column groups per row block
  int nfc1;               // workgroups with fc1 tiles: nrb * ngrp
  const float* X;         // [S * M, K1] this launch's inputs (cut activations), row-major
  const int64_t* Y;       // [S * M] labels
  float* loss;            // [S * M] per-row losses
  int64_t ignore;
  float ce_scale;         // per-row loss scale (1 / M)
  SlOpt o;                // kind / lr / betas / eps / wd / momentum (step scalars: adam)
  const float* adam;      // [S][4] {step_size, inv_bc2_sqrt, CE scale (1 / the step's rows), -}
  const uint32_t* seeds;  // [S][4] {fc1 lo, hi, fc2 lo, hi} dropout seeds per step
  uint32_t thr1, thr2;    // dropout thresholds (0: off)
  float dsc1, dsc2;       // 1 / (1 - p)
  int col_off1;           // global index of this shard's fc1 row 0 (dropout hash column)
  int lookahead_last;     // 1: the last step also forms the next batch's fc1 product (unused: 0)
  // hand-off buffers (zeroed once by the host; double-buffered by step parity)
  float* LA;              // [2][ngrp][16][N1p] fc1 look-ahead partial pre-activations
  float* H1;              // [2][16][N1p] h1 rows published by each row block's last-arriving column group
  float* LP;              // [2][G][16][C4] logit partials of each workgroup's fc2 rows
  float* DL;              // [2][16][C4] dlogits
  float* DZ2;             // [2][16][G][4] fc2 output gradient, dz2[m][w + G ii] at [m][w][ii]
  float* W2B;             // [2][nrb][G][16][4] W2 after each step: W2[w + G ii][16 rb + jj] at [rb][w][jj][ii]
  unsigned* cnt;          // [kResCounters][kResShardStride] arrival counters (zeroed per launch)
  const int* shard_n;     // [kResSeams][8] arrivals per shard and step
  int* err;               // nonzero after a wait gave up (timeout or a peer's error)
  int64_t timeout;        // wall-clock ticks per wait
  // tensor-parallel fc2 (row-parallel): the peer-mapped exchange of each workgroup's fc2
  // product rows; ipc.T == 0: single shard
  IpcStep ipc;
  // optional phase timestamps (wall clock) of workgroups 0 and G - 1 for the first
  // trace_steps steps: [2][trace_steps][16] (scripts/resident_trace.py)
  int64_t* trace;
  int trace_steps;
  // 1: cooperative launch (the runtime refuses a grid the device cannot hold at once); 0: a
  // plain launch, for ranks that deliberately share one GPU with a partial grid each (the
  // one-GPU multi-process rehearsal), where the device-wide check does not describe the split
  int coop;
  int fault_step;         // fault injection (tests): this step's first wait is never met (times out, err 2); -1: off
};

hipError_t resident_epoch_launch(const ResArgs& a, hipStream_t st);
// Workgroups the launch needs and whether the device keeps them all resident at once.
int resident_lds_bytes(const ResArgs& a);
bool resident_fits(const ResArgs& a, int device, std::string* why);

}  // namespace sl
