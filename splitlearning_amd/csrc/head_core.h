// The U-shape head step (reference model3 = Linear(100, 10) + CrossEntropyLoss on Alice,
// data_entities.py:74-81) for M <= 16 rows, C <= 16 classes, K <= 128 (% 4) features, as a
// device function of one 256-thread workgroup: shared by `head_step_mfma_kernel` (loss.hip,
// its own launch) and `ushape_mid_kernel` (ushape.hip, behind Bob's middle in the same
// launch).  The three products run on exact-fp32 MFMA (v_mfma_f32_16x16x4f32, 16 x 16 tiles):
// logits (wave 0, K / 4 steps), data gradient (one 16-column tile of K per wave step, C
// padded to 16) and weight gradient (M = 16 as the reduction); the softmax-CE on DPP row
// reductions over the 16 class lanes of each row.  bf16 compute is a template parameter.
#pragma once
#include "common.h"

namespace sl {

struct HeadLds {
  static constexpr int KP = 132;   // padded LDS row (K <= 128)
  float sx[16][KP];                // X, zero-padded to 16 rows
  float sw[16][KP];                // W [C][K], zero-padded to 16 classes
  float sg[16][KP];                // dW [C][K]
  float sd[16][17];                // dlogits [M][C]
};

// The head's operands that do not depend on X: the optimizer state of W and b, b and W
// itself (head_preload), loaded before X exists when the caller can (ushape_mid_kernel issues
// them before it knows whether it is the workgroup that runs the head).
struct HeadPre {
  static constexpr int PF = 8;     // state elements per thread (C K <= 2048)
  float r0[PF], r1[PF];
  float rb0, rb1, rbp;
  f32x4 wr[2];
};

__device__ __forceinline__ void head_preload(HeadPre& P, const float* __restrict__ W, const float* __restrict__ bias,
                                             const float* __restrict__ s0w, const float* __restrict__ s1w,
                                             const float* __restrict__ s0b, const float* __restrict__ s1b, int K,
                                             int C) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < HeadPre::PF; ++j) {
    const int i = tid + 256 * j;
    P.r0[j] = i < C * K ? s0w[i] : 0.f;
    P.r1[j] = (i < C * K && s1w) ? s1w[i] : 0.f;
  }
  P.rb0 = P.rb1 = P.rbp = 0.f;
  if (bias && tid < C) {
    P.rbp = bias[tid];
    P.rb0 = s0b[tid];
    P.rb1 = s1b ? s1b[tid] : 0.f;
  }
  const int K4 = K >> 2;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int f = tid + 256 * j, r = f / K4;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    P.wr[j] = r < C ? reinterpret_cast<const f32x4*>(W)[f] : z4;
  }
}

// x_staged: the caller already wrote X (rows < M, columns < K; zeros elsewhere) into L.sx and
// synchronised; otherwise X is read from global memory.  Every thread of the workgroup calls
// this (it synchronises); threads >= 256 must not exist.
template <bool BF>
__device__ __forceinline__ void head_core(HeadLds& L, const HeadPre& P, bool x_staged, const float* __restrict__ X,
                                          const float* __restrict__ bias, const int64_t* __restrict__ y,
                                          int64_t ignore, float scale, float* __restrict__ loss_rows,
                                          float* __restrict__ dX, float* __restrict__ Wout, float* __restrict__ bout,
                                          float* __restrict__ s0w, float* __restrict__ s1w, float* __restrict__ s0b,
                                          float* __restrict__ s1b, int M, int K, int C, SlOpt o, int mask_dx) {
  constexpr int KP = HeadLds::KP;
  auto R = [](float v) { return BF ? bfr(v) : v; };
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lq = lane >> 4;
  constexpr int PF = HeadPre::PF;
  const int K4 = K >> 2;
  f32x4 xr[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int f = tid + 256 * j, r = f / K4;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    xr[j] = (!x_staged && r < M) ? reinterpret_cast<const f32x4*>(X)[f] : z4;
  }
  for (int i = tid; i < 16 * KP; i += 256) {
    if (!x_staged) (&L.sx[0][0])[i] = 0.f;
    (&L.sw[0][0])[i] = 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int f = tid + 256 * j, r = f / K4, q = f - r * K4;
    if (r < 16) {
      if (!x_staged) *reinterpret_cast<f32x4*>(&L.sx[r][4 * q]) = xr[j];
      *reinterpret_cast<f32x4*>(&L.sw[r][4 * q]) = P.wr[j];
    }
  }
  __syncthreads();
  // logits D[m][c] = sum_k X[m][k] W[c][k] (wave 0): A lane (m = li, k = 4s + lq), B (k, c = li)
  if (wv == 0) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s4 = 0; s4 < K; s4 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(R(L.sx[li][s4 + lq]), R(L.sw[li][s4 + lq]), acc, 0, 0, 0);
    // lane (c = li, lq) holds rows m = 4 lq + r; softmax over the 16 class lanes of each row
    const bool vc = li < C;
    const float bc = (bias && vc) ? bias[li] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * lq + r;
      const float z = vc ? acc[r] + bc : -INFINITY;
      const float mx = sl_row16_max(z);
      const float e = vc ? expf(z - mx) : 0.f;
      const float se = sl_row16_sum(e);
      float dl = 0.f;
      if (m < M) {
        const int64_t lab = y[m];
        if (lab == ignore) {
          if (li == 0) loss_rows[m] = 0.f;
        } else {
          const float zl = sl_dpp_pick(z, (int)lab);
          if (li == 0) loss_rows[m] = mx + logf(se) - zl;
          if (vc) dl = (e / se - (li == lab ? 1.f : 0.f)) * scale;
        }
      }
      L.sd[m][li] = dl;
    }
  }
  __syncthreads();
  // data gradient dX[m][k] = sum_c dlog[m][c] W[c][k]: wave w takes 16-column tiles w, w+4, ..
  for (int kt = wv; kt * 16 < K; kt += 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(R(L.sd[li][s4 + lq]), R(L.sw[s4 + lq][16 * kt + li]), acc, 0, 0, 0);
    const int k = 16 * kt + li;
    if (k < K) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * lq + r;
        if (m < M) dX[m * K + k] = (mask_dx && !(L.sx[m][k] > 0.f)) ? 0.f : acc[r];
      }
    }
  }
  // weight gradient dW[c][k] = sum_m dlog[m][c] X[m][k] -> LDS
  for (int kt = wv; kt * 16 < K; kt += 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(R(L.sd[s4 + lq][li]), R(L.sx[s4 + lq][16 * kt + li]), acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) L.sg[4 * lq + r][16 * kt + li] = acc[r];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int i = tid + 256 * j;
    if (i < C * K) {
      const int c = i / K, k = i - c * K;
      float pp = L.sw[c][k], a0 = P.r0[j], a1 = P.r1[j];
      sl_opt_update(o, pp, L.sg[c][k], a0, a1);
      if (o.kind != 0) Wout[i] = pp;
      s0w[i] = a0;
      if (s1w) s1w[i] = a1;
    }
  }
  if (bias && tid < C) {
    float g = 0.f;
    for (int m = 0; m < M; ++m) g += L.sd[m][tid];
    float pp = P.rbp, a0 = P.rb0, a1 = P.rb1;
    sl_opt_update(o, pp, g, a0, a1);
    if (o.kind != 0) bout[tid] = pp;
    s0b[tid] = a0;
    if (s1b) s1b[tid] = a1;
  }
}

}  // namespace sl
