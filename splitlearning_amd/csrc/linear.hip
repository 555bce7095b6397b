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

hipError_t gemm_nt(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K, Epi e,
                   bool bf16, hipStream_t st);

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
template <int U>
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
    const int kk = kb + 16 * u + kq;
    const bool in = kk < K;                      // K % 4 == 0: a float4 never straddles K
    a[u] = (va && in) ? ld4(pa + kk) : z4;
    w[u] = (vb && in) ? ld4(pb + kk) : z4;
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    acc0 = mfma4(a[u].x, w[u].x, acc0);
    acc1 = mfma4(a[u].y, w[u].y, acc1);
    acc0 = mfma4(a[u].z, w[u].z, acc0);
    acc1 = mfma4(a[u].w, w[u].w, acc1);
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
  // waves per workgroup (variant 14: 3 -> 4, 4 -> 16, for A/B; default 8)
  const int nwt = g_variant[14] == 3 ? 4 : (g_variant[14] == 4 ? 16 : 8);
  NW = std::min(waves, nwt);
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
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_t pack_bf16x8(float4 lo, float4 hi) {
  bf16x8_t v;
  v[0] = (__bf16)lo.x; v[1] = (__bf16)lo.y; v[2] = (__bf16)lo.z; v[3] = (__bf16)lo.w;
  v[4] = (__bf16)hi.x; v[5] = (__bf16)hi.y; v[6] = (__bf16)hi.z; v[7] = (__bf16)hi.w;
  return v;
}

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

// Full-N dgrad: dX[M, K] = mask(dZ[M, N] . W[N, K]) with the WHOLE reduction over N inside
// one workgroup, so the result is stored masked and final (no split-N slabs, no reduce
// launch).  grid (ceil(K/32), ceil(M/16)), 1024 threads = 16 waves; wave w owns an N slice.
// MFMA v_mfma_f32_16x16x4f32 with A = dZ (16 rows m x 4 n), B = W (4 n x 16 k): the 32
// k-columns of the workgroup are two 16-column MFMA tiles fed by one float2 load per lane
// (16 lanes x 8 B = one 128-B row segment of W per n).  Lane (m = lane&15, q = lane>>4) takes
// n = n0 + 4q + s at sub-step s, so its four dZ values of a 16-n group are one float4 load.
// The 16 waves' partial tiles are summed through LDS in a fixed order (deterministic).
// At B = 16 this reads W once (fc2: 20 MB) from 157 workgroups; the split-N form it replaces
// needed ~630 workgroups plus a reduce launch over the slabs.
template <int NC>   // columns per lane: 2 (32-column tiles, float2 loads) or 1 (16-column tiles)
__global__ void __launch_bounds__(1024)
dgrad_fulln_kernel(const float* __restrict__ dZ, int ldz, const float* __restrict__ W, int ldw,
                   const float* __restrict__ hprev, int ldh, float scale, float* __restrict__ out, int ldo,
                   int M, int N, int K) {
  __shared__ f32x4 red[16][NC][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int k0 = blockIdx.x * 16 * NC, m0 = blockIdx.y * 16;
  const int j = lane & 15, q = lane >> 4;
  const int kc = k0 + NC * j;                      // this lane's NC columns kc ..
  const bool vk = kc + NC - 1 < K;                 // K % 4 == 0 (host check): never straddles K
  const bool vm = (m0 + j) < M;
  // N slice of this wave: multiples of 16
  const int nper = ((N + 16 * 16 - 1) / (16 * 16)) * 16;
  const int nb = wv * nper, ne = min(N, nb + nper);
  const float* za = dZ + (int64_t)(vm ? m0 + j : 0) * ldz;
  f32x4 acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto ldw_ = [&](int nn) {
    float2 r = make_float2(0.f, 0.f);
    if (NC == 2)
      r = *reinterpret_cast<const float2*>(W + (int64_t)nn * ldw + kc);
    else
      r.x = W[(int64_t)nn * ldw + kc];
    return r;
  };
  constexpr int U = 4;                             // 16-n groups in flight per lane
  int n = nb;
  for (; n + 16 * U <= ne; n += 16 * U) {
    float4 a[U];
    float2 w[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int nq = n + 16 * u + 4 * q;
      a[u] = vm ? *reinterpret_cast<const float4*>(za + nq) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int s = 0; s < 4; ++s) w[u][s] = vk ? ldw_(nq + s) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float av[4] = {a[u].x, a[u].y, a[u].z, a[u].w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc[0] = mfma4(av[s], w[u][s].x, acc[0]);
        if (NC == 2) acc[NC - 1] = mfma4(av[s], w[u][s].y, acc[NC - 1]);
      }
    }
  }
  for (; n < ne; n += 16) {                        // tail groups (N % 16 handled per element)
    const int nq = n + 4 * q;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int nn = nq + s;
      const bool in = nn < ne;
      const float av = (vm && in) ? za[nn] : 0.f;
      const float2 wv2 = (vk && in) ? ldw_(nn) : make_float2(0.f, 0.f);
      acc[0] = mfma4(av, wv2.x, acc[0]);
      if (NC == 2) acc[NC - 1] = mfma4(av, wv2.y, acc[NC - 1]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[wv][c][lane] = acc[c];
  __syncthreads();
  // 256 NC outputs: thread t -> (column half h, lane l); D_h[row][col]: row = 4*(l>>4) + r, col j = l & 15
  const int t = threadIdx.x;
  if (t < 64 * NC) {
    const int h = t >> 6, l = t & 63;
    f32x4 sm = red[0][h][l];
#pragma unroll
    for (int v = 1; v < 16; ++v) sm += red[v][h][l];
    const int kk = k0 + NC * (l & 15) + h;
    if (kk < K) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 4 * (l >> 4) + r;
        if (m >= M) continue;
        float v = sm[r];
        if (hprev) v = (hprev[(int64_t)m * ldh + kk] > 0.f) ? v * scale : 0.f;
        out[(int64_t)m * ldo + kk] = v;
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
  if (M > 128) return gemm_nt(X, ldx, W, ldw, Y, ldy, M, N, K, e, g_bf16 != 0, st);
  dim3 grid((N + 15) / 16, (M + 15) / 16);
  int NW1, S1;
  if (!g_bf16 && g_variant[14] != 2 && fwd_once_plan(M, N, K, 16, ws ? ws_elems : 0, NW1, S1)) {
    skinny_fwd_once_kernel<4><<<dim3(grid.x, grid.y, S1), NW1 * 64, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, ws,
                                                                          (int64_t)M * N);
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
  // variant 8 = 2: the full-N form (reduction over N inside one workgroup, masked store, one
  // launch).  Measured through the native executor it LOST to the split-N + reduce pair
  // below at every TP shard (us per server step, TP = 1 / 2 / 4 / 8: 171.9 / 104.4 / 72.5 /
  // 55.6 full-N vs 170.9 / 101.6 / 68.9 / 51.8 split; profiles/r2_dgrad_fulln_ab.txt): with
  // the whole N per workgroup there are only K/32 workgroups (20 at a TP = 8 shard), each a
  // chain of 1000-row strided reads, and the reduce launch is cheaper than that latency.
  // variant 8 = 3: the same with 16-column tiles (twice the workgroups, one float per lane):
  // also slower than the split pair, us per step at TP = 1 / 2 / 4 / 8: 179.2 / 103.2 / 70.8 /
  // 54.6 vs 176.8 / 101.0 / 68.5 / 51.8 (profiles/r2_dgrad_fulln16_ab.txt).
  if ((g_variant[8] == 2 || g_variant[8] == 3) && !g_bf16 && M <= 64 && (K & 3) == 0 && (ldw & 1) == 0 &&
      (ldz & 3) == 0) {
    if (g_variant[8] == 3) {
      dgrad_fulln_kernel<1><<<dim3((K + 15) / 16, mt), 1024, 0, st>>>(dZ, ldz, W, ldw, hprev, ldh, scale, dX, ldx, M,
                                                                       N, K);
    } else {
      dgrad_fulln_kernel<2><<<dim3((K + 31) / 32, mt), 1024, 0, st>>>(dZ, ldz, W, ldw, hprev, ldh, scale, dX, ldx, M,
                                                                       N, K);
    }
    return hipGetLastError();
  }
  int S = 1;
  // aim for >= ~256 workgroups on the 256-CU part; split N when there are few K tiles.
  // Variant 5, for A/B: 1 = never split, >1 = max split with N slices down to 16 rows.
  // Both measured slower or equal at every TP shard (at TP = 8: 57.6 us per native-executor
  // server step unsplit vs 51.8 us split; profiles/r1_dgrad_split_ab.txt).
  const int v5 = g_variant[5];
  const int smax = v5 > 0 ? v5 : 16;
  // few K tiles over a long N (a TP shard's fc2: K = 628, N = 1000 at TP = 8): N slices down
  // to 32 rows (S = 16): 3.1 vs 3.7 us per launch in the graph-replay probe
  // (scripts/probe/dgrad_probe.hip).  Short N (the U-shape fc2, N = 100) stays unsplit: one
  // launch with the mask fused beats a split plus a reduce launch.
  const int rmin = v5 > 1 ? 16 : ((kt * mt <= 64 && N >= 512) ? 32 : 64);
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
    // TP = 1, S = 16 at a TP = 8 shard; variant 19 = 2: plain order)
    const int nblk = ((N + 4 * S - 1) / (4 * S)) * 4;
    const int xg = (g_variant[19] != 2 && S % 8 == 0 && nblk * (S / 8) == 128) ? S / 8 : 0;
    if (g_bf16)
      skinny_dgrad_kernel<8, true><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, 0, slab, M, N, K, xg);
    else
      skinny_dgrad_kernel<8><<<grid, 512, 0, st>>>(dZ, ldz, W, ldw, nullptr, 0, 1.f, ws, 0, slab, M, N, K, xg);
    launch_dgrad_reduce(ws, S, slab, hprev, ldh, scale, dX, ldx, M, K, st);
  }
  return hipGetLastError();
}

// fc1's look-ahead epilogue fused into fc2's split-K forward (single-shard tail, variant 18
// = 1).  Workgroup (ks, nr, mt) owns the 64-wide k-slice ks of h1 for 16 rows: it reduces
// the S1 look-ahead slabs of that slice in slab order (bitwise the epilogue kernel's sum),
// applies fc1's bias / ReLU / dropout (writing h1 when nr == 0), stages the tile in LDS and
// forms the slice's partial product with fc2's 128 output columns nr on exact-fp32 MFMA;
// P2 gets one slab per k-slice for the head to reduce.  The W2 loads are issued first, so
// they overlap the slab reduction.  The k-slice runs fastest in the grid, padded to a
// multiple of 8, so the 8 column ranges of one slice share an XCD (and its L2 copy of the
// slabs).  Removes the epilogue launch — and measured slower through the native executor
// (us per TP = 1 step, profiles/r2_lookahead_fc2_fused_ab.txt): 173.0 (64-wide slices) and
// 176.5 (128-wide) vs 170.8 for the epilogue + split-K forward pair.  The slab round trip now
// sits in front of every workgroup's MFMAs, and the head reduces 79 / 40 product slabs
// instead of the forward's 16: more latency than the launch boundary it saves.  Opt-in.
template <int LKS>
__global__ void __launch_bounds__(256)
lookahead_fc2_fwd_kernel(const float* __restrict__ pn, int S1, int64_t slab1, Epi e1, float* __restrict__ h1,
                         const float* __restrict__ W2, float* __restrict__ P2, int64_t slab2, int M, int N1, int N2,
                         int nks) {
  __shared__ float At[16][LKS + 4];
  const int ks = blockIdx.x;
  if (ks >= nks) return;                                 // grid padding (XCD grouping)
  const int nr = blockIdx.y, m0 = blockIdx.z * 16, k0 = ks * LKS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q4 = (lane >> 4) * 4, j = lane & 15;
  constexpr int U = LKS / 16;
  // W2 rows of this wave's two 16-column tiles: every load before anything else
  float4 w[2][U];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = (nr * 8 + 2 * wv + t) * 16 + j;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k0 + 16 * u + q4;
      w[t][u] = (n < N2 && kk < N1) ? ld4(W2 + (int64_t)n * N1 + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // h1 tile: thread -> (row r, float4 columns c4, c4 + 16, ...); the slabs summed in order
  // from 0
  const int r = tid >> 4;
#pragma unroll
  for (int c4 = tid & 15; c4 < LKS / 4; c4 += 16) {
    const int m = m0 + r, k = k0 + 4 * c4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m < M && k < N1) {
      const float* p = pn + (int64_t)m * N1 + k;
      constexpr int SU = 32;
      for (int s0 = 0; s0 < S1; s0 += SU) {
        float4 rr[SU];
#pragma unroll
        for (int i = 0; i < SU; ++i)
          rr[i] = (s0 + i < S1) ? ld4(p + (int64_t)(s0 + i) * slab1) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < SU; ++i) v += f32x4{rr[i].x, rr[i].y, rr[i].z, rr[i].w};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = apply_epi(e1, v[i], m, k + i);
      if (nr == 0) *reinterpret_cast<f32x4*>(h1 + (int64_t)m * N1 + k) = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) At[r][4 * c4 + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n0 = (nr * 8 + 2 * wv + t) * 16;
    if (n0 >= N2) break;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* ar = &At[j][16 * u + q4];
      acc0 = mfma4(ar[0], w[t][u].x, acc0);
      acc1 = mfma4(ar[1], w[t][u].y, acc1);
      acc0 = mfma4(ar[2], w[t][u].z, acc0);
      acc1 = mfma4(ar[3], w[t][u].w, acc1);
    }
    const f32x4 sm = acc0 + acc1;
    const int n = n0 + j;
    if (n < N2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + q4 + r;
        if (m < M) P2[(int64_t)ks * slab2 + (int64_t)m * N2 + n] = sm[r];
      }
    }
  }
}

// k-slice width: variant 18 = 1 -> 64, = 2 -> 128
static int lookahead_ks() { return g_variant[18] == 2 ? 128 : 64; }
int lookahead_fc2_slices(int N1) { return (N1 + 63) / 64; }   // capacity bound (the narrower slice)

hipError_t lookahead_fc2_fwd(const float* pn, int S1, int64_t slab1, Epi e1, float* h1, const float* W2, float* P2,
                             int64_t p2_elems, int M, int N1, int N2, int* S2_out, hipStream_t st) {
  *S2_out = 0;
  if (M <= 0) return hipSuccess;
  const int ks = lookahead_ks();
  const int nks = (N1 + ks - 1) / ks;
  if ((N1 & 3) || S1 < 1 || (int64_t)nks * M * N2 > p2_elems) return hipErrorInvalidValue;
  const dim3 g((nks + 7) / 8 * 8, (N2 + 127) / 128, (M + 15) / 16);
  if (ks == 128)
    lookahead_fc2_fwd_kernel<128><<<g, 256, 0, st>>>(pn, S1, slab1, e1, h1, W2, P2, (int64_t)M * N2, M, N1, N2, nks);
  else
    lookahead_fc2_fwd_kernel<64><<<g, 256, 0, st>>>(pn, S1, slab1, e1, h1, W2, P2, (int64_t)M * N2, M, N1, N2, nks);
  *S2_out = nks;
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
  if (!g_bf16 && g_variant[14] != 2 && fwd_once_plan(M, N, K, max_split, ws_elems, NW1, S1)) {
    Epi e1{};
    e1.dscale = 1.f;
    // XCD-grouped tile order (at most 64 column tiles: grid padded to 64); variant 19 = 2:
    // plain order.  Native executor, us per TP = 1 step: 174.4 vs 175.5 and 176.9 vs 178.1 in
    // two interleaved runs (profiles/r2_xcd_grouped_fc2_ab.txt); bitwise the same products.
    const bool xg = g_variant[19] != 2 && grid.x <= 64;
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
