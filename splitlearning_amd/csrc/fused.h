// Descriptors shared by the fused server-step kernels (fused.hip) and the bindings.
#pragma once
#include "common.h"
#include "ipc_ar.h"

namespace sl {

struct WgDesc {
  const float* dz;      // [M, N] output gradient (ld ldz)
  int ldz;
  const float* A;       // [M, K] layer input
  int lda;
  float* W;
  int ldw;
  float* s0;
  float* s1;
  float* bias;
  float* sb0;
  float* sb1;
  int N, K;
  int yb0;              // first blockIdx.y of this layer (2-D grid)
  int wb0;              // first block of this layer (1-D grid)
};
struct WgGroup {
  WgDesc d[3];
  int n;
  // Optional look-ahead forward of layer 0 with its *updated* weights:
  //   pn[kb][m][n] = sum_{k in k-block kb} xn[m, k] * W0_new[n, k]   (kb = 256-column blocks)
  // i.e. the next batch's split-K partial pre-activations, written while W0 is in registers.
  const float* xn;      // [mn, K0] next batch input (mn <= 64), or nullptr
  int ldxn;
  int mn;
  float* pn;            // [ceil(K0/256)][mn][N0]
  int rev0;             // walk layer 0's tiles last-to-first (set by wgrad_group)
  int nt0;              // layer 0's tile count (set by wgrad_group)
  int grid2d;           // 2-D grid (set by wgrad_group: when few of its workgroups are empty)
  int wt;               // write-through (sc1) W/m/v stores (set by wgrad_group)
  int bf16;             // bf16 compute: dZ / A / look-ahead operands rounded to bf16 (set by wgrad_group)
  int afirst;           // load the first chunk's A / dZ before W / m / v (set by wgrad_group)
  int pol;              // W / state load and store cache policy preset (set by wgrad_group; variant 21)
  int rt;               // row tiles per workgroup of the streaming form (set by wgrad_group; 0 = tiled form)
  int pin;              // streaming form: layer-0 rows [0, pin) plain both ways, the rest non-temporal (variant 23)
};

int head3_slices(int N2);
// head_fwd + head_bwd (fused.hip).  ipc (tensor-parallel fc2): P2 is this rank's unreduced
// [M, N2] partial; the head pushes its slice
// to every rank, waits for the T slices and sums them in rank order (the fc2 all-reduce fused
// into the slab reduction: ipc_ar.h).  G > 1: the C logits are G cross-entropy groups (labels
// y [M, G], per-(row, group) scales gscale [M, G] or `scale`, losses loss_rows [M, G]).
hipError_t server_head3(const float* P2, int S2, int64_t slab2, Epi e2, const float* W3, int ldw3, const float* b3,
                        const int64_t* y, int64_t ignore, float scale, float* h2, float* dlog, float* dz2,
                        float* loss_rows, float* ws, int64_t ws_elems, int M, int N2, int C, hipStream_t st,
                        const IpcStep* ipc = nullptr, int G = 1, const float* gscale = nullptr);
hipError_t wgrad_group(const WgGroup& g, int M, SlOpt o, hipStream_t st);

}  // namespace sl
