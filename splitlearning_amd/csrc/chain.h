// The server step's latency chain in ONE launch (csrc/chain.hip): between two wgrad_group
// launches, the launch-per-stage executor (engine.cpp) issues six short kernels (fc1 epilogue,
// fc2 forward, head_fwd, head_bwd, fc2 dgrad, dgrad reduce), ~36 us of a 173 us TP = 1 step
// (profiles/r3q_bench_n1_kernel_summary.txt) that move ~50 MB.  chain_step_launch runs the
// same math as one persistent launch with in-launch hand-offs (the seams of resident.hip).
#pragma once
#include "common.h"
#include "ipc_ar.h"

#include <string>

namespace sl {

constexpr int kChThreads = 512;      // 8 waves, one workgroup per CU
constexpr int kChRB = 8;             // fc2 row blocks of the W2 tiles (<= 128 rows each)
constexpr int kChMaxCB = 32;         // fc2 column blocks (<= 40 float4 each)
constexpr int kChMaxWR = 128;        // tile rows
constexpr int kChMaxWC4 = 40;        // tile columns / 4
constexpr int kChMaxC = 128;         // classes
constexpr int kChMaxSlabs = 24;      // fc1 look-ahead slabs (fc1 input width <= 6144)
constexpr int kChSeams = 4;          // 0: fc2 partials, 1: logit partials, 2: dlogits, 3: dz2
constexpr int kChStride = 32;        // counter words between counters (128 B)
constexpr int kChCounters = kChSeams * 8 + 2 * kChMaxCB;   // seam shards, then 2 sets of column-group counters

struct ChainArgs {
  int M, N1, N2, C, C4;
  int G, NCB, HW;             // workgroups, column blocks (tiles = kChRB * NCB), head workgroups (N2 / 4)
  // fc1: pending look-ahead slabs of the step's batch, [S1][M][N1] (slab stride `slab`)
  const float* pn;
  int S1;
  int64_t slab;
  Epi e1;                     // fc1 bias + ReLU + dropout
  float s1;                   // fc1 dropout scale for dz1 (1 / (1 - p1))
  const float* W2;            // [N2][N1]
  Epi e2;                     // fc2 bias + ReLU + dropout
  const float* W3;            // [C][N2]
  const float* b3;            // [C]
  const int64_t* Y;           // [M] labels
  int64_t ignore;
  float ce_scale;
  // outputs (the wgrad launch's operands)
  float *h1, *h2, *dlog, *dz2, *dz1, *loss;
  // hand-offs
  float* FP;                  // [NCB][16][N2] fc2 product partials per column block
  float* LP;                  // [HW][16][C4] logit partials per head workgroup
  float* DL;                  // [16][C4] dlogits (C4 pitch)
  float* DP;                  // [kChRB][16][N1] dz1 partials per row block
  unsigned* cnt;              // [kChCounters][kChStride], zeroed once per epoch
  const int* shard_n;         // [kChSeams][8] arrivals per shard and launch
  unsigned gen;               // launches since the counters were zeroed, 1-based
  int* err;                   // nonzero once a wait gave up
  int64_t timeout;            // wall-clock ticks per wait
  IpcStep ipc;                // tensor-parallel fc2: the peer-mapped exchange (T == 0: none)
  int64_t* trace;             // optional: phase wall-clock stamps of workgroups 0 and G - 1, [2][16]
};

// Whether the shapes fit the kernel's tiles (empty string) or why not.
std::string chain_check(const ChainArgs& a);
// Workgroups the device keeps co-resident (0 if the kernel cannot run).
int chain_max_workgroups(int device);
hipError_t chain_step_launch(const ChainArgs& a, hipStream_t st);

}  // namespace sl
