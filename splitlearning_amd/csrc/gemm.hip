// LDS-tiled MFMA GEMM for many rows: Y[M, N] = epi(X[M, K] . W[N, K]^T).
//
// Reference op: nn.Linear (models.py:36-37,49-53,69-73,90) on a whole batch of rows — Bob's
// inference over a client's test set in evaluation (the reference scores 16-row batches
// over RPC, data_entities_vanilla.py:172-178; here one call per client) and large
// `--batch_size` training batches.  The skinny kernels (linear.hip) cover M <= 128, where
// streaming W is the bound; past that the product is compute-bound and this kernel tiles it:
//
//  * 128 x 128 output tile per 256-thread workgroup, 2 x 2 waves of 64 x 64, each wave a
//    4 x 4 grid of 16 x 16 MFMA blocks (16 accumulators of 4 floats);
//  * fp32: exact-fp32 v_mfma_f32_16x16x4_f32, K staged 16 at a time; a lane reads ONE float4
//    of its A row and of its B row per stage and feeds its component j to sub-step j (the
//    four lane groups q cover k = 4q + j), so A/B fragments are single ds_read_b128s;
//  * bf16 (`--dtype bf16`): operands rounded to bf16 (RNE, v_cvt_pk_bf16_f32) as they are
//    staged, v_mfma_f32_16x16x32_bf16 with fp32 accumulation, K staged 32 at a time;
//  * double-buffered LDS: the next stage's global loads are issued before this stage's
//    MFMAs, written to the other buffer after them (one barrier per stage);
//  * epilogue (bias + ReLU + counter-hash dropout, common.h apply_epi) fused into the store.
// Rows are padded (fp32 +4 floats, bf16 +8 halves) so the 16 rows a lane group reads land on
// different banks.  Requires K % 4 == 0 and 16-byte aligned rows (host checks).
#include "common.h"

#include <type_traits>

namespace sl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <bool BF16>
struct GemmCfg {
  static constexpr int BK = BF16 ? 32 : 16;      // K per stage
  static constexpr int LD = BF16 ? 40 : 20;      // LDS row stride (elements, padded)
  typedef typename std::conditional<BF16, __bf16, float>::type T;
};

__device__ __forceinline__ bf16x4 to_bf16x4(float4 v) {
  bf16x4 o;
  o[0] = (__bf16)v.x;
  o[1] = (__bf16)v.y;
  o[2] = (__bf16)v.z;
  o[3] = (__bf16)v.w;
  return o;
}

template <bool BF16>
__global__ void __launch_bounds__(256)
gemm_nt_kernel(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw, float* __restrict__ Y,
               int ldy, int M, int N, int K, Epi e) {
  using C = GemmCfg<BF16>;
  using T = typename C::T;
  constexpr int BK = C::BK, LD = C::LD;
  constexpr int PER = 128 * BK / 4 / 256;          // float4 loads per thread per operand per stage (2 / 4)
  constexpr int TPR = BK / 4;                       // threads per row in a load pass (4 / 8)
  constexpr int RPP = 256 / TPR;                    // rows per load pass (64 / 32)
  __shared__ __attribute__((aligned(16))) T As[2][128][LD];
  __shared__ __attribute__((aligned(16))) T Bs[2][128][LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // XCD-aware tile order: consecutive workgroups (dealt round-robin over the 8 XCDs) walk
  // down M for one N column strip, so the strip of W a tile reads is shared through the
  // Infinity Cache while X rows stream
  const int tilesM = (M + 127) / 128;
  const int tm = blockIdx.x % tilesM, tn = blockIdx.x / tilesM;
  const int m0 = tm * 128, n0 = tn * 128;
  const int lr = tid / TPR, lk = (tid % TPR) * 4;
  float4 ra[PER], rb[PER];
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int r = lr + p * RPP, k = k0 + lk;
      const int gm = m0 + r, gn = n0 + r;
      ra[p] = (gm < M && k < K) ? *reinterpret_cast<const float4*>(X + (int64_t)gm * ldx + k) : z4;
      rb[p] = (gn < N && k < K) ? *reinterpret_cast<const float4*>(W + (int64_t)gn * ldw + k) : z4;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int r = lr + p * RPP;
      if constexpr (BF16) {
        *reinterpret_cast<bf16x4*>(&As[buf][r][lk]) = to_bf16x4(ra[p]);
        *reinterpret_cast<bf16x4*>(&Bs[buf][r][lk]) = to_bf16x4(rb[p]);
      } else {
        *reinterpret_cast<float4*>(&As[buf][r][lk]) = ra[p];
        *reinterpret_cast<float4*>(&Bs[buf][r][lk]) = rb[p];
      }
    }
  };
  const int wm = (wv & 1) * 64, wn = (wv >> 1) * 64;
  const int li = lane & 15, lq = lane >> 4;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) gload((s + 1) * BK);        // next stage's loads in flight during the MFMAs
    if constexpr (BF16) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = *reinterpret_cast<const bf16x8*>(&As[buf][wm + 16 * i + li][8 * lq]);
        b[i] = *reinterpret_cast<const bf16x8*>(&Bs[buf][wn + 16 * i + li][8 * lq]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    } else {
      f32x4 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = *reinterpret_cast<const f32x4*>(&As[buf][wm + 16 * i + li][4 * lq]);
        b[i] = *reinterpret_cast<const f32x4*>(&Bs[buf][wn + 16 * i + li][4 * lq]);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][c], b[j][c], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nk) {
      sstore(buf ^ 1);    // the other buffer: its last readers finished before the previous barrier
      __syncthreads();
    }
  }
  // epilogue: lane (li, lq) of block (i, j) holds rows 4 lq + r, column li
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + 16 * j + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * lq + r;
        if (m < M) Y[(int64_t)m * ldy + n] = apply_epi(e, acc[i][j][r], m, n);
      }
    }
}

hipError_t gemm_nt(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K, Epi e,
                   bool bf16, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if ((K & 3) || (ldx & 3) || (ldw & 3)) return hipErrorInvalidValue;
  const int64_t tiles = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  if (bf16)
    gemm_nt_kernel<true><<<(unsigned)tiles, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e);
  else
    gemm_nt_kernel<false><<<(unsigned)tiles, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e);
  return hipGetLastError();
}

}  // namespace sl
