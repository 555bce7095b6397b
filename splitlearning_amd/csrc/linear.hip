// Skinny Linear-layer kernels for Bob's server tail and the U-shape head.
//
// Reference ops: nn.Linear fc1/fc2/fc3 (models.py:36-37,49-53,69-73,90) with the
// ReLU / Dropout(0.5) that follow them, trained by SGD-m (vanilla,
// data_entities_vanilla.py:37-42) or Adam (U-shape data_entities.py:43-47; SISA
// Adam(wd=1e-5) data_entities_vanilla_sisa.py:266).  SURVEY §2.7 K5-K8, K11-K12.
//
// Shape regime: M = batch (16 by default) rows against weights of up to
// 5000 x 5408 (108 MB fp32).  At M = 16 every kernel is bound by streaming the
// weight / optimizer state through HBM, so the design goal is bytes, not FLOPs:
//   * forward  Y = X W^T: exact-fp32 MFMA (v_mfma_f32_16x16x4_f32), one 16-column
//     tile per workgroup, the workgroup's waves split K and reduce through LDS,
//     bias + ReLU + dropout fused in the epilogue (no second pass over Y);
//   * dgrad    dX = dZ W: same MFMA, a 64-column K tile per workgroup, waves split
//     N, optional split-N across workgroups, ReLU/dropout backward of the *previous*
//     layer fused into the store;
//   * wgrad + optimizer: dW is never materialised.  A 1024-thread workgroup owns a
//     16-row x 256-column tile, each thread one float4 of a row; g = sum_m dZ[m,n] X[m,k]
//     from LDS-staged operands, then SGD-momentum / Adam in place: 24 B of HBM traffic
//     per parameter (p, m, v read + write) instead of 36 B for wgrad-then-optimizer.
//   Variants that measured slower (non-temporal loads, software-pipelined forward,
//   row-blocked and loads-first wgrad) were removed after measurement (docs/PERF.md).
#include "common.h"

#include <algorithm>

namespace sl {

int g_variant[24] = {0};
int g_bf16 = 0;
int g_nn_splits = 0;
int g_nn_wm = 0;
int g_nt_splits = 0;

hipError_t gemm_nt(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K, Epi e,
                   bool bf16, float* ws, int64_t ws_elems, hipStream_t st);

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }



// ---------------------------------------------------------------------------- forward
// grid (ceil(N/16), ceil(M/16)), block NW*64.  Requires K % 4 == 0, ldx/ldw % 4 == 0.
// U = float4 pairs in flight per lane per iteration; NT = non-temporal weight loads
// (every weight is read by exactly one wave once per step, so keep it out of L2).
// Split-K (gridDim.z = S > 1): workgroup z covers its own 16-aligned slice of K and stores
// raw partial sums to P[z][M][N]; epilogue_kernel then reduces the S slabs and applies the
// epilogue.  Splitting K is what balances the load: the fc1 GEMM has only 313 column
// tiles for 256 CUs, and each CU's load issue rate (16 rows x 64 B per wave instruction)
// is the limiter, so ~4 workgroups per CU beat 1-2 big ones.
template <int NW, int U, bool NT>
__global__ void __launch_bounds__(NW * 64)
skinny_fwd_kernel(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw,
                  float* __restrict__ Y, int ldy, int M, int N, int K, Epi e,
                  float* __restrict__ P = nullptr, int64_t slab = 0) {
  __shared__ f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16;
  const int S = gridDim.z;
  const int kz = ((K + 16 * S - 1) / (16 * S)) * 16;
  const int kz0 = min(K, (int)blockIdx.z * kz), kz1 = min(K, kz0 + kz);
  const int kper = ((kz1 - kz0 + 16 * NW - 1) / (16 * NW)) * 16;
  const int kb = kz0 + wv * kper;
  const int ke = min(kz1, kb + kper);
  const int ra = m0 + (lane & 15), rb = n0 + (lane & 15);
  const int kq = (lane >> 4) * 4;
  const bool va = ra < M, vb = rb < N;
  const float* pa = X + (int64_t)(va ? ra : 0) * ldx;
  const float* pb = W + (int64_t)(vb ? rb : 0) * ldw;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  int k = kb;
  // main loop: 16*U k per iteration, U independent float4 pairs in flight per lane
  for (; k + 16 * U <= ke; k += 16 * U) {
    float4 a[U];
    f32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = va ? ld4(pa + k + 16 * u + kq) : z4;
      if (NT)
        w[u] = vb ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(pb + k + 16 * u + kq)) : zv;
      else
        w[u] = vb ? *reinterpret_cast<const f32x4*>(pb + k + 16 * u + kq) : zv;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc0 = mfma4(a[u].x, w[u][0], acc0);
      acc1 = mfma4(a[u].y, w[u][1], acc1);
      acc0 = mfma4(a[u].z, w[u][2], acc0);
      acc1 = mfma4(a[u].w, w[u][3], acc1);
    }
  }
  for (; k < ke; k += 16) {
    const int kk = k + kq;
    const bool in = kk < ke;
    float4 a = (va && in) ? ld4(pa + kk) : z4;
    float4 w = (vb && in) ? ld4(pb + kk) : z4;
    acc0 = mfma4(a.x, w.x, acc0);
    acc1 = mfma4(a.y, w.y, acc1);
    acc0 = mfma4(a.z, w.z, acc0);
    acc1 = mfma4(a.w, w.w, acc1);
  }
  red[wv][lane] = acc0 + acc1;
  __syncthreads();
  if (wv == 0) {
    f32x4 s = red[0][lane];
#pragma unroll
    for (int i = 1; i < NW; ++i) s += red[i][lane];
    const int n = n0 + (lane & 15);
    if (n < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + (lane >> 4) * 4 + r;
        if (m >= M) continue;
        if (S == 1)
          Y[(int64_t)m * ldy + n] = apply_epi(e, s[r], m, n);
        else
          P[(int64_t)blockIdx.z * slab + (int64_t)m * N + n] = s[r];
      }
    }
  }
}

// One-round-trip form (the default; variant 14 = 2 selects skinny_fwd_kernel): every wave
// owns exactly 16 U consecutive k of its 16-column tile and issues ALL its loads (U float4 of
// X and of W per lane) before the first MFMA, so a wave costs one memory round trip; the
// workgroup is NW = blockDim / 64 waves (NW 16 U k per split-K slice), summed through LDS in
// wave order.  skinny_fwd_kernel walks its k range in dependent U-batches (at fc2's shape, K =
// 5000 in 16 slices of 320 k over 2 waves, 4 round trips per wave).  Native executor, us per
// server step (profiles/r2_chain_probe.txt): TP = 1 177.8 vs 178.1 and 174.9 vs 175.3, TP = 8
// 52.3 vs 53.0 and 53.2 vs 53.9 — small, but the same sign in both interleaved runs.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_t pack_bf16x8(float4 lo, float4 hi) {
  bf16x8_t v;
  v[0] = (__bf16)lo.x; v[1] = (__bf16)lo.y; v[2] = (__bf16)lo.z; v[3] = (__bf16)lo.w;
  v[4] = (__bf16)hi.x; v[5] = (__bf16)hi.y; v[6] = (__bf16)hi.z; v[7] = (__bf16)hi.w;
  return v;
}

// BF: `--dtype bf16` form — lane group q stages k = 8q .. 8q + 7 of each 32-k step (two float4 of
// its X row and W row, the fp32 form's bytes) for one v_mfma_f32_16x16x32_bf16 per step.
template <int U, bool BF = false>
__global__ void __launch_bounds__(1024)
skinny_fwd_once_kernel(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw,
                       float* __restrict__ Y, int ldy, int M, int N, int K, Epi e, float* __restrict__ P,
                       int64_t slab, int nt_real = 0) {
  __shared__ f32x4 red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, NW = blockDim.x >> 6;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (nt_real > 0) {
    // XCD-grouped order (default; variant 19 = 2 off; grid x padded to 64 column tiles): dispatch slot L
    // goes to XCD L % 8 (round robin), and every slot of XCD g takes a column tile of the
    // 128 W rows [128 g, 128 g + 128), so one XCD's L2 holds those rows for the fc2 dgrad
    // that follows (skinny_dgrad_kernel, same grouping).  Tile math and sums unchanged.
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int j = L >> 3;
    bx = 8 * (L & 7) + (j & 7);
    by = (j >> 3) % gridDim.y;
    bz = (j >> 3) / gridDim.y;
    if (bx >= nt_real) return;
  }
  const int n0 = bx * 16, m0 = by * 16;
  const int S = gridDim.z;
  const int kb = (bz * NW + wv) * 16 * U;
  const int ra = m0 + (lane & 15), rb = n0 + (lane & 15);
  const int kq = (lane >> 4) * 4;
  const bool va = ra < M, vb = rb < N;
  const float* pa = X + (int64_t)(va ? ra : 0) * ldx;
  const float* pb = W + (int64_t)(vb ? rb : 0) * ldw;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 a[U], w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    // fp32: 16-k steps, lane group q at k = 4q; bf16: 32-k steps, lane group q at k = 8q, 8q + 4
    const int kk = BF ? kb + 32 * (u >> 1) + 2 * kq + 4 * (u & 1) : kb + 16 * u + kq;
    const bool in = kk < K;                      // K % 4 == 0: a float4 never straddles K
    a[u] = (va && in) ? ld4(pa + kk) : z4;
    w[u] = (vb && in) ? ld4(pb + kk) : z4;
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (BF) {
#pragma unroll
    for (int u = 0; u < U; u += 2)
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pack_bf16x8(a[u], a[u + 1]), pack_bf16x8(w[u], w[u + 1]), acc0,
                                                     0, 0, 0);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc0 = mfma4(a[u].x, w[u].x, acc0);
      acc1 = mfma4(a[u].y, w[u].y, acc1);
      acc0 = mfma4(a[u].z, w[u].z, acc0);
      acc1 = mfma4(a[u].w, w[u].w, acc1);
    }
  }
  red[wv][lane] = acc0 + acc1;
  __syncthreads();
  if (wv == 0) {
    f32x4 s = red[0][lane];
    for (int i = 1; i < NW; ++i) s += red[i][lane];
    const int n = n0 + (lane & 15);
    if (n < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + (lane >> 4) * 4 + r;
        if (m >= M) continue;
        if (S == 1)
          Y[(int64_t)m * ldy + n] = apply_epi(e, s[r], m, n);
        else
          P[(int64_t)bz * slab + (int64_t)m * N + n] = s[r];
      }
    }
  }
}

// Launch plan of skinny_fwd_once_kernel (U = 4: 64 k per wave): NW waves per workgroup and S
// split-K slices with S <= max_split and S M N <= ws_elems (S == 1 needs no workspace).
// Returns false when K does not fit (the caller keeps skinny_fwd_kernel).
static bool fwd_once_plan(int M, int N, int K, int max_split, int64_t ws_elems, int& NW, int& S) {
  constexpr int KW = 64;
  const int waves = (K + KW - 1) / KW;            // waves per 16 x 16 output tile
  const int64_t slab = (int64_t)M * N;
  const int64_t fit = ws_elems / (slab > 0 ? slab : 1);
  const int smax = (int)std::max<int64_t>(1, std::min<int64_t>(max_split, fit));
  // a product that one 16-wave workgroup per tile covers (K <= 1024: the U-shape fc2, a TP
  // shard's fc2) runs unsplit, so the epilogue is fused and no slab-reduce launch follows
  if (waves <= 16) {
    NW = waves;
    S = 1;
    return true;
  }
  // 8 waves per workgroup (4 and 16 measured no better, docs/PERF.md)
  NW = std::min(waves, 8);
  S = (waves + NW - 1) / NW;
  if (S > smax) {
    S = smax;
    NW = (waves + S - 1) / S;
  }
  return NW <= 16;
}

// bf16 compute form of skinny_fwd_kernel (`--dtype bf16`): same grid, split-K and store, but
// each lane stages 8 consecutive k of its X row and W row (two float4 loads each), rounds
// them to bf16 and issues one v_mfma_f32_16x16x32_bf16 (lane group q covers k = 8q..8q+7 of
// a 32-k step); fp32 accumulation.  K slices are 32-aligned.
template <int NW, int U>
__global__ void __launch_bounds__(NW * 64)
skinny_fwd_bf16_kernel(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw,
                       float* __restrict__ Y, int ldy, int M, int N, int K, Epi e,
                       float* __restrict__ P = nullptr, int64_t slab = 0) {
  __shared__ f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16;
  const int S = gridDim.z;
  const int kz = ((K + 32 * S - 1) / (32 * S)) * 32;
  const int kz0 = min(K, (int)blockIdx.z * kz), kz1 = min(K, kz0 + kz);
  const int kper = ((kz1 - kz0 + 32 * NW - 1) / (32 * NW)) * 32;
  const int kb = kz0 + wv * kper;
  const int ke = min(kz1, kb + kper);
  const int ra = m0 + (lane & 15), rb = n0 + (lane & 15);
  const int kq = (lane >> 4) * 8;
  const bool va = ra < M, vb = rb < N;
  const float* pa = X + (int64_t)(va ? ra : 0) * ldx;
  const float* pb = W + (int64_t)(vb ? rb : 0) * ldw;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  int k = kb;
  for (; k + 32 * U <= ke; k += 32 * U) {
    float4 a0[U], a1[U], w0[U], w1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k + 32 * u + kq;
      a0[u] = va ? ld4(pa + kk) : z4;
      a1[u] = va ? ld4(pa + kk + 4) : z4;
      w0[u] = vb ? ld4(pb + kk) : z4;
      w1[u] = vb ? ld4(pb + kk + 4) : z4;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pack_bf16x8(a0[u], a1[u]), pack_bf16x8(w0[u], w1[u]), acc, 0, 0, 0);
  }
  for (; k < ke; k += 32) {
    const int kk = k + kq;
    const bool i0 = kk < ke, i1 = kk + 4 < ke;
    const float4 a0 = (va && i0) ? ld4(pa + kk) : z4, a1 = (va && i1) ? ld4(pa + kk + 4) : z4;
    const float4 w0 = (vb && i0) ? ld4(pb + kk) : z4, w1 = (vb && i1) ? ld4(pb + kk + 4) : z4;
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pack_bf16x8(a0, a1), pack_bf16x8(w0, w1), acc, 0, 0, 0);
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv == 0) {
    f32x4 s = red[0][lane];
#pragma unroll
    for (int i = 1; i < NW; ++i) s += red[i][lane];
    const int n = n0 + (lane & 15);
    if (n < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + (lane >> 4) * 4 + r;
        if (m >= M) continue;
        if (S == 1)
          Y[(int64_t)m * ldy + n] = apply_epi(e, s[r], m, n);
        else
          P[(int64_t)blockIdx.z * slab + (int64_t)m * N + n] = s[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------- dgrad
// dX[M,K] = dZ[M,N] . W[N,K]; grid (ceil(K/64), ceil(M/16), S), block NW*64.
// S == 1: store with the fused mask (h_prev > 0) * scale.  S > 1: store raw partial
// sums to P[s][M][K] (reduced by dgrad_reduce_kernel).  Requires K % 4 == 0.
template <int NW, bool BF = false>
__global__ void __launch_bounds__(NW * 64)
skinny_dgrad_kernel(const float* __restrict__ dZ, int ldz, const float* __restrict__ W, int ldw,
                    const float* __restrict__ hprev, int ldh, float scale,
                    float* __restrict__ out, int ldo, int64_t slab, int M, int N, int K, int xcd8 = 0) {
  __shared__ f32x4 red[NW][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (xcd8) {
    // XCD-grouped order (default; S = 8 xcd8 slices, xcd8 of them per 128-row group): dispatch
    // slot L goes to XCD L % 8 and takes an N slice of row group L % 8, i.e. the W rows the
    // forward's XCD-grouped order left in that XCD's L2 (skinny_fwd_once_kernel).  Tile math
    // and sums unchanged.
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int j = L >> 3;
    bz = (L & 7) * xcd8 + j % xcd8;
    bx = (j / xcd8) % gridDim.x;
    by = (j / xcd8) / gridDim.x;
  }
  const int k0 = bx * 64, m0 = by * 16;
  const int S = gridDim.z, sidx = bz;
  // N range for this workgroup, then for this wave (multiples of 4)
  const int nblk = ((N + 4 * S - 1) / (4 * S)) * 4;
  const int nb0 = sidx * nblk, ne0 = min(N, nb0 + nblk);
  const int nper = (((ne0 - nb0) + 4 * NW - 1) / (4 * NW)) * 4;
  const int nb = nb0 + wv * nper;
  const int ne = min(ne0, nb + nper);
  const int i = lane & 15, q = lane >> 4;
  const int kcol = k0 + 4 * i;
  const bool vk = kcol < K;
  const bool vm = (m0 + i) < M;
  const float* za = dZ + (int64_t)(vm ? m0 + i : 0) * ldz;
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = {0.f, 0.f, 0.f, 0.f};
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  int n = nb;
  if (BF) {
    // bf16 MFMA (v_mfma_f32_16x16x16_bf16), k index = n: lane (i, q) supplies dZ[m0 + i][n + 4q ..
    // n + 4q + 3] (one float4) and, per column c of its float4, W[n + 4q .. n + 4q + 3][kcol + c]
    // (four row loads: the fp32 form's bytes per 16 rows), so one MFMA per column group
    // replaces four exact-fp32 ones; the accumulator layout is the fp32 form's.
    typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
    for (; n + 16 <= ne; n += 16) {
      const int nq = n + 4 * q;
      const float4 a4 = vm ? ld4(za + nq) : z4;
      float4 wr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) wr[r] = vk ? ld4(W + (int64_t)(nq + r) * ldw + kcol) : z4;
      const bf16x4_t A = {(__bf16)a4.x, (__bf16)a4.y, (__bf16)a4.z, (__bf16)a4.w};
      const bf16x4_t B0 = {(__bf16)wr[0].x, (__bf16)wr[1].x, (__bf16)wr[2].x, (__bf16)wr[3].x};
      const bf16x4_t B1 = {(__bf16)wr[0].y, (__bf16)wr[1].y, (__bf16)wr[2].y, (__bf16)wr[3].y};
      const bf16x4_t B2 = {(__bf16)wr[0].z, (__bf16)wr[1].z, (__bf16)wr[2].z, (__bf16)wr[3].z};
      const bf16x4_t B3 = {(__bf16)wr[0].w, (__bf16)wr[1].w, (__bf16)wr[2].w, (__bf16)wr[3].w};
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A, B0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A, B1, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A, B2, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A, B3, acc[3], 0, 0, 0);
    }
  }
  for (; n + 16 <= ne; n += 16) {
    float a[4];
    float4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int nn = n + 4 * u + q;
      a[u] = vm ? za[nn] : 0.f;
      w[u] = vk ? ld4(W + (int64_t)nn * ldw + kcol) : z4;
      if (BF) {
        a[u] = bfr(a[u]);
        w[u] = bfr4(w[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0] = mfma4(a[u], w[u].x, acc[0]);
      acc[1] = mfma4(a[u], w[u].y, acc[1]);
      acc[2] = mfma4(a[u], w[u].z, acc[2]);
      acc[3] = mfma4(a[u], w[u].w, acc[3]);
    }
  }
  for (; n < ne; n += 4) {
    const int nn = n + q;
    const bool vn = nn < ne;
    float a = (vm && vn) ? za[nn] : 0.f;
    float4 w = (vk && vn) ? ld4(W + (int64_t)nn * ldw + kcol) : z4;
    if (BF) {
      a = bfr(a);
      w = bfr4(w);
    }
    acc[0] = mfma4(a, w.x, acc[0]);
    acc[1] = mfma4(a, w.y, acc[1]);
    acc[2] = mfma4(a, w.z, acc[2]);
    acc[3] = mfma4(a, w.w, acc[3]);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) red[wv][c][lane] = acc[c];
  __syncthreads();
  // 4 waves finish: wave c' reduces column-group c' (needs NW >= 4)
  if (wv < 4) {
    const int c = wv;
    f32x4 s = red[0][c][lane];
#pragma unroll
    for (int v = 1; v < NW; ++v) s += red[v][c][lane];
    // D_c[row][j]: row = (lane>>4)*4 + r, j = lane & 15 -> k = k0 + 4j + c
    const int kk = k0 + 4 * (lane & 15) + c;
    if (kk < K) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + (lane >> 4) * 4 + r;
        if (m >= M) continue;
        float v = s[r];
        if (S == 1) {
          if (hprev) v = (hprev[(int64_t)m * ldh + kk] > 0.f) ? v * scale : 0.f;
          out[(int64_t)m * ldo + kk] = v;
        } else {
          out[(int64_t)sidx * slab + (int64_t)m * K + kk] = v;
        }
      }
    }
  }
}

__global__ void dgrad_reduce_kernel(const float* __restrict__ P, int S, int64_t slab,
                                    const float* __restrict__ hprev, int ldh, float scale,
                                    float* __restrict__ out, int ldo, int M, int K) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)M * K) return;
  const int m = (int)(t / K), k = (int)(t - (int64_t)m * K);
  float v = sum_slabs(P + t, S, slab);
  if (hprev) v = (hprev[(int64_t)m * ldh + k] > 0.f) ? v * scale : 0.f;
  out[(int64_t)m * ldo + k] = v;
}

// Y = epilogue(P) for a GEMM done elsewhere (large-M eval path): P [M,N] with ld ldp.
__global__ void epilogue_kernel(const float* __restrict__ P, int ldp, float* __restrict__ Y, int ldy,
                                int M, int N, Epi e, int S = 1, int64_t slab = 0) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)M * N) return;
  const int m = (int)(t / N), n = (int)(t - (int64_t)m * N);
  const float v = sum_slabs(P + (int64_t)m * ldp + n, S, slab);
  Y[(int64_t)m * ldy + n] = apply_epi(e, v, m, n);
}

// The slab reductions stay scalar (one column per thread): float4 forms (4 columns per
// thread, 256- or 64-thread workgroups) won a graph-replay probe with the slabs L2-hot
// (scripts/probe/dgrad_probe.hip: 2.0 vs 2.7 us) but lost 0.3-1.5 us per server step in the
// native executor at every TP degree (profiles/r2_chain_probe.txt): with the slabs cold, a
// quarter of the threads is a quarter of the loads in flight.
static void launch_epilogue(const float* P, int ldp, float* Y, int ldy, int M, int N, Epi e, int S, int64_t slab,
                            hipStream_t st) {
  const int64_t tot = (int64_t)M * N;
  epilogue_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(P, ldp, Y, ldy, M, N, e, S, slab);
}

static void launch_dgrad_reduce(const float* P, int S, int64_t slab, const float* hprev, int ldh, float scale,
                                float* out, int ldo, int M, int K, hipStream_t st) {
  const int64_t tot = (int64_t)M * K;
  dgrad_reduce_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(P, S, slab, hprev, ldh, scale, out, ldo, M, K);
}

// the split-K reduction + ReLU / dropout mask of a data gradient computed elsewhere (gemm.hip)
hipError_t dgrad_reduce(const float* P, int S, int64_t slab, const float* hprev, int ldh, float scale, float* out,
                        int ldo, int M, int K, hipStream_t st) {
  if (M <= 0 || K <= 0) return hipSuccess;
  launch_dgrad_reduce(P, S, slab, hprev, ldh, scale, out, ldo, M, K, st);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- wgrad + optimizer
// v3: memory-level parallelism first.  A 1024-thread workgroup owns a 16-row x 256-column
// tile; every wave covers one row's 256 contiguous weights (1 KB per instruction), so each
// thread holds exactly one float4 of p/m/v, issues those loads before anything else, and
// stays at ~40 VGPRs (32 waves/CU resident).  The tile's 16x256 slice of A and its 16x16
// slice of dZ are staged once in LDS and shared by all 16 rows (A re-read from L2 once
// per 16 rows); the per-thread dot product is 16 broadcast-free ds_read_b128 + 64 FMAs.
template <bool ADAM>
__global__ void __launch_bounds__(1024)
wgrad_opt_v3_kernel(const float* __restrict__ dZ, int ldz, const float* __restrict__ A, int lda,
                    float* __restrict__ W, int ldw, float* __restrict__ s0, float* __restrict__ s1,
                    float* __restrict__ bias, float* __restrict__ sb0, float* __restrict__ sb1,
                    int M, int N, int K, SlOpt o, int g_bf) {
  __shared__ f32x4 sa[16][64];
  __shared__ float sdz[16][16];
  const int tid = threadIdx.x;
  const int r = tid >> 6, lane = tid & 63;
  const int n = blockIdx.y * 16 + r;
  const int k = blockIdx.x * 256 + lane * 4;
  const bool act = (n < N) && (k < K);
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  const int64_t off = (int64_t)n * ldw + k;
  f32x4 p = zv, q0 = zv, q1 = zv;
  if (act) {
    p = *reinterpret_cast<const f32x4*>(W + off);
    q0 = *reinterpret_cast<const f32x4*>(s0 + off);
    if (ADAM) q1 = *reinterpret_cast<const f32x4*>(s1 + off);
  }
  f32x4 g = zv;
  float gb = 0.f;
  for (int mc = 0; mc < M; mc += 16) {
    if (mc) __syncthreads();
    {
      const int m = mc + r, kk = blockIdx.x * 256 + lane * 4;
      const f32x4 av = (m < M && kk < K) ? *reinterpret_cast<const f32x4*>(A + (int64_t)m * lda + kk) : zv;
      sa[r][lane] = g_bf ? bfr4(av) : av;
      if (tid < 256) {
        const int mm = mc + (tid >> 4), nn = blockIdx.y * 16 + (tid & 15);
        const float dv = (mm < M && nn < N) ? dZ[(int64_t)mm * ldz + nn] : 0.f;
        sdz[tid >> 4][tid & 15] = g_bf ? bfr(dv) : dv;
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const float d = sdz[m][r];
      g += d * sa[m][lane];
      gb += d;
    }
  }
  if (act) {
    sl_opt_update4<ADAM>(o, p, g, q0, q1);
    if (o.kind != 0) *reinterpret_cast<f32x4*>(W + off) = p;
    *reinterpret_cast<f32x4*>(s0 + off) = q0;
    if (ADAM) *reinterpret_cast<f32x4*>(s1 + off) = q1;
  }
  if (bias && blockIdx.x == 0 && lane == 0 && n < N) {
    float pb = bias[n], b0 = sb0[n], b1 = sb1 ? sb1[n] : 0.f;
    sl_opt_update(o, pb, gb, b0, b1);
    if (o.kind != 0) bias[n] = pb;
    sb0[n] = b0;
    if (sb1) sb1[n] = b1;
  }
}

// Plain elementwise optimizer over a flat parameter (generic fallback / tests).
__global__ void opt_flat_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ s0,
                                float* __restrict__ s1, int64_t n, SlOpt o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float pp = p[i], a0 = s0[i], a1 = s1 ? s1[i] : 0.f;
  sl_opt_update(o, pp, g[i], a0, a1);
  if (o.kind != 0) p[i] = pp;
  s0[i] = a0;
  if (s1) s1[i] = a1;
}

// ---------------------------------------------------------------------------- host launchers
hipError_t linear_fwd(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N,
                      int K, Epi e, float* ws, int64_t ws_elems, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  // many rows (evaluation over a whole test set, large batches): the LDS-tiled MFMA GEMM.
  // In fp32 the caller (hip_ops.linear_fwd) hands plain products to hipBLASLt and only the
  // epilogue runs here, except inside a HIP graph capture or under variant 11 = 1.
  if (M > 128) return gemm_nt(X, ldx, W, ldw, Y, ldy, M, N, K, e, g_bf16 != 0, ws, ws_elems, st);
  dim3 grid((N + 15) / 16, (M + 15) / 16);
  int NW1, S1;
  if (fwd_once_plan(M, N, K, 16, ws ? ws_elems : 0, NW1, S1)) {
    if (g_bf16)
      skinny_fwd_once_kernel<4, true><<<dim3(grid.x, grid.y, S1), NW1 * 64, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K,
                                                                                  e, ws, (int64_t)M * N);
    else
      skinny_fwd_once_kernel<4><<<dim3(grid.x, grid.y, S1), NW1 * 64, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e,
                                                                            ws, (int64_t)M * N);
    if (S1 > 1) {
      launch_epilogue(ws, N, Y, ldy, M, N, e, S1, (int64_t)M * N, st);
    }
    return hipGetLastError();
  }
  // split K until there are ~8 workgroups per CU, keeping >= 256 k per workgroup: fc1
  // (313 column tiles) runs S = 4 (30.6 us vs 35.2 us at S = 2; profiles/r1_kbench_call17)
  const int tiles = grid.x * grid.y;
  int S = 1;
  while (S < 16 && tiles * S * 2 <= 2048 && K / (S * 2) >= 256) S *= 2;
  const int64_t slab = (int64_t)M * N;
  if (S > 1 && (ws == nullptr || ws_elems < slab * S)) S = 1;
  const int kz = (K + S - 1) / S;
  const int nw = kz >= 1024 ? 8 : (kz >= 512 ? 4 : 2);
  dim3 g3(grid.x, grid.y, S);
  float* P = S > 1 ? ws : nullptr;
  if (g_bf16) {
    if (nw == 8)
      skinny_fwd_bf16_kernel<8, 2><<<g3, 512, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, P, slab);
    else if (nw == 4)
      skinny_fwd_bf16_kernel<4, 2><<<g3, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, P, slab);
    else
      skinny_fwd_bf16_kernel<2, 2><<<g3, 128, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, P, slab);
  } else if (nw == 8)
    skinny_fwd_kernel<8, 4, false><<<g3, 512, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, P, slab);
  else if (nw == 4)
    skinny_fwd_kernel<4, 4, false><<<g3, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, P, slab);
  else
    skinny_fwd_kernel<2, 4, false><<<g3, 128, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, P, slab);
  if (S > 1) {
    launch_epilogue(ws, N, Y, ldy, M, N, e, S, slab, st);
  }
  return hipGetLastError();
}

hipError_t linear_dgrad(const float* dZ, int ldz, const float* W, int ldw, const float* hprev, int ldh,
                        float scale, float* dX, int ldx, float* ws, int64_t ws_elems, int M, int N, int K,
                        hipStream_t st) {
  if (M <= 0 || K <= 0) return hipSuccess;
  const int kt = (K + 63) / 64, mt = (M + 15) / 16;
  // A full-N form (the whole reduction over N in one workgroup, masked store, one launch)
  // LOST to this split-N + reduce pair at every TP shard (us per server step, TP = 1 / 2 / 4 /
  // 8: 171.9 / 104.4 / 72.5 / 55.6 vs 170.9 / 101.6 / 68.9 / 51.8; profiles/r2_dgrad_fulln_ab.txt):
  // only K/32 workgroups, each a chain of strided reads.  Removed in round 3 (git history).
  int S = 1;
  // aim for >= ~256 workgroups on the 256-CU part; split N when there are few K tiles.
  // Never splitting measured slower at every TP shard (TP = 8: 57.6 vs 51.8 us per native
  // server step; profiles/r1_dgrad_split_ab.txt).
  const int smax = 16;
  // few K tiles over a long N (a TP shard's fc2: K = 628, N = 1000 at TP = 8): N slices down
  // to 32 rows (S = 16): 3.1 vs 3.7 us per launch in the graph-replay probe
  // (scripts/probe/dgrad_probe.hip).  Short N (the U-shape fc2, N = 100) stays unsplit: one
  // launch with the mask fused beats a split plus a reduce launch.
  const int rmin = (kt * mt <= 64 && N >= 512) ? 32 : 64;
  while (S < smax && kt * mt * S < 768 && N / (S * 2) >= rmin) S *= 2;
  const int64_t slab = (int64_t)M * K;
  if (ws == nullptr) S = 1;
  while (S > 1 && ws_elems < slab * S) S >>= 1;
  dim3 grid(kt, mt, S);
  if (S == 1) {
    if (g_bf16)
      skinny_dgrad_kernel<8, true><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, hprev, ldh, scale, dX, ldx, 0, M, N, K);
    else
      skinny_dgrad_kernel<8><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, hprev, ldh, scale, dX, ldx, 0, M, N, K);
  } else {
    // XCD-grouped order when S / 8 N slices make one 128-row group of the forward (S = 8 at
    // TP = 1, S = 16 at a TP = 8 shard)
    const int nblk = ((N + 4 * S - 1) / (4 * S)) * 4;
    const int xg = (S % 8 == 0 && nblk * (S / 8) == 128) ? S / 8 : 0;
    if (g_bf16)
      skinny_dgrad_kernel<8, true><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, 0, slab, M, N, K, xg);
    else
      skinny_dgrad_kernel<8><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, 0, slab, M, N, K, xg);
    launch_dgrad_reduce(ws, S, slab, hprev, ldh, scale, dX, ldx, M, K, st);
  }
  return hipGetLastError();
}

// Partial-output variants for fused consumers (server_head3 / wgrad_group reduce the slabs
// themselves): the split-K (fwd) or split-N (dgrad) slabs, or the plain product when no
// split is chosen, land in ws as [S][M][cols]; *S_out receives S.
hipError_t linear_fwd_partial(const float* X, int ldx, const float* W, int ldw, int M, int N, int K, float* ws,
                              int64_t ws_elems, int max_split, int* S_out, hipStream_t st) {
  *S_out = 1;
  if (M <= 0 || N <= 0) return hipSuccess;
  dim3 grid((N + 15) / 16, (M + 15) / 16);
  const int tiles = grid.x * grid.y;
  int S = 1;
  while (S < max_split && tiles * S * 2 <= 2048 && K / (S * 2) >= 256) S *= 2;
  const int64_t slab = (int64_t)M * N;
  if (ws_elems < slab * S) S = 1;
  if (ws_elems < slab) return hipErrorInvalidValue;
  int NW1, S1;
  if (fwd_once_plan(M, N, K, max_split, ws_elems, NW1, S1)) {
    Epi e1{};
    e1.dscale = 1.f;
    // XCD-grouped tile order (at most 64 column tiles: grid padded to 64).  Native executor,
    // us per TP = 1 step against the plain order: 174.4 vs 175.5 and 176.9 vs 178.1 in two
    // interleaved runs (profiles/r2_xcd_grouped_fc2_ab.txt); bitwise the same products.
    const bool xg = grid.x <= 64;
    if (g_bf16)
      skinny_fwd_once_kernel<4, true><<<dim3(xg ? 64 : grid.x, grid.y, S1), NW1 * 64, 0, st>>>(
          X, ldx, W, ldw, ws, N, M, N, K, e1, ws, slab, xg ? (int)grid.x : 0);
    else
      skinny_fwd_once_kernel<4><<<dim3(xg ? 64 : grid.x, grid.y, S1), NW1 * 64, 0, st>>>(
          X, ldx, W, ldw, ws, N, M, N, K, e1, ws, slab, xg ? (int)grid.x : 0);
    *S_out = S1;
    return hipGetLastError();
  }
  const int kz = (K + S - 1) / S;
  const int nw = kz >= 1024 ? 8 : (kz >= 512 ? 4 : 2);
  dim3 g3(grid.x, grid.y, S);
  Epi e{};
  e.dscale = 1.f;
  if (g_bf16) {
    if (nw == 8)
      skinny_fwd_bf16_kernel<8, 2><<<g3, 512, 0, st>>>(X, ldx, W, ldw, ws, N, M, N, K, e, ws, slab);
    else if (nw == 4)
      skinny_fwd_bf16_kernel<4, 2><<<g3, 256, 0, st>>>(X, ldx, W, ldw, ws, N, M, N, K, e, ws, slab);
    else
      skinny_fwd_bf16_kernel<2, 2><<<g3, 128, 0, st>>>(X, ldx, W, ldw, ws, N, M, N, K, e, ws, slab);
  } else if (nw == 8)
    skinny_fwd_kernel<8, 4, false><<<g3, 512, 0, st>>>(X, ldx, W, ldw, ws, N, M, N, K, e, ws, slab);
  else if (nw == 4)
    skinny_fwd_kernel<4, 4, false><<<g3, 256, 0, st>>>(X, ldx, W, ldw, ws, N, M, N, K, e, ws, slab);
  else
    skinny_fwd_kernel<2, 4, false><<<g3, 128, 0, st>>>(X, ldx, W, ldw, ws, N, M, N, K, e, ws, slab);
  *S_out = S;
  return hipGetLastError();
}

hipError_t linear_dgrad_partial(const float* dZ, int ldz, const float* W, int ldw, int M, int N, int K, float* ws,
                                int64_t ws_elems, int* S_out, hipStream_t st) {
  *S_out = 1;
  if (M <= 0 || K <= 0) return hipSuccess;
  const int kt = (K + 63) / 64, mt = (M + 15) / 16;
  int S = 1;
  while (S < 16 && kt * mt * S < 768 && N / (S * 2) >= 64) S *= 2;
  const int64_t slab = (int64_t)M * K;
  if (ws_elems < slab * S) S = 1;
  if (ws_elems < slab) return hipErrorInvalidValue;
  dim3 grid(kt, mt, S);
  if (g_bf16)
    skinny_dgrad_kernel<8, true><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, S == 1 ? K : 0,
                                                        S == 1 ? 0 : slab, M, N, K);
  else if (S == 1)
    skinny_dgrad_kernel<8><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, K, 0, M, N, K);
  else
    skinny_dgrad_kernel<8><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, 0, slab, M, N, K);
  *S_out = S;
  return hipGetLastError();
}

hipError_t linear_epilogue(const float* P, int ldp, float* Y, int ldy, int M, int N, Epi e, int S, int64_t slab,
                           hipStream_t st) {
  if ((int64_t)M * N <= 0) return hipSuccess;
  launch_epilogue(P, ldp, Y, ldy, M, N, e, S, slab, st);
  return hipGetLastError();
}

hipError_t linear_wgrad_opt(const float* dZ, int ldz, const float* A, int lda, float* W, int ldw, float* s0,
                            float* s1, float* bias, float* sb0, float* sb1, int M, int N, int K, SlOpt o,
                            hipStream_t st) {
  if (N <= 0 || K <= 0) return hipSuccess;
  // v3 layout (5.8 TB/s effective on fc1 at M = 16)
  dim3 g3((K + 255) / 256, (N + 15) / 16);
  if (o.kind == 2)
    wgrad_opt_v3_kernel<true><<<g3, 1024, 0, st>>>(dZ, ldz, A, lda, W, ldw, s0, s1, bias, sb0, sb1, M, N, K, o,
                                                    g_bf16);
  else
    wgrad_opt_v3_kernel<false><<<g3, 1024, 0, st>>>(dZ, ldz, A, lda, W, ldw, s0, s1, bias, sb0, sb1, M, N, K, o,
                                                     g_bf16);
  return hipGetLastError();
}

hipError_t opt_flat(float* p, const float* g, float* s0, float* s1, int64_t n, SlOpt o, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  opt_flat_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(p, g, s0, s1, n, o);
  return hipGetLastError();
}

}  // namespace sl
