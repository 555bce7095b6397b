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

__device__ __forceinline__ bf16x4 to_bf16x4(float4 v) {
  bf16x4 o;
  o[0] = (__bf16)v.x;
  o[1] = (__bf16)v.y;
  o[2] = (__bf16)v.z;
  o[3] = (__bf16)v.w;
  return o;
}

// WM: waves along M (the workgroup is WM x 2 waves, each a 64 x 64 output tile, so the tile is
// 64 WM x 128); BK: K per LDS stage (fp32: 16 or 32; bf16: 32 or 64).
template <bool BF16, int WM, int BK>
__global__ void __launch_bounds__(128 * WM)
gemm_nt_kernel(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw, float* __restrict__ Y,
               int ldy, int M, int N, int K, Epi e) {
  using T = typename std::conditional<BF16, __bf16, float>::type;
  constexpr int BM = 64 * WM, BN = 128, NT = 128 * WM;
  constexpr int LD = BK + (BF16 ? 8 : 4);           // padded LDS row (elements)
  constexpr int F4R = BK / 4;                        // float4s per row per stage
  constexpr int APER = BM * F4R / NT, BPER = BN * F4R / NT;
  static_assert(APER * NT == BM * F4R && BPER * NT == BN * F4R, "tile / thread split");
  static_assert(!BF16 || BK % 32 == 0, "bf16 stages are whole 16x16x32 MFMA steps");
  __shared__ __attribute__((aligned(16))) T As[2][BM][LD];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN][LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // tiles of one N column strip are consecutive workgroups: the strip of W is read by many
  // tiles back to back (served from L2 / the Infinity Cache) while X rows stream
  const int tilesM = (M + BM - 1) / BM;
  const int tm = blockIdx.x % tilesM, tn = blockIdx.x / tilesM;
  const int m0 = tm * BM, n0 = tn * BN;
  float4 ra[APER], rb[BPER];
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = k0 + (i % F4R) * 4, gm = m0 + r;
      ra[p] = (gm < M && k < K) ? *reinterpret_cast<const float4*>(X + (int64_t)gm * ldx + k) : z4;
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = k0 + (i % F4R) * 4, gn = n0 + r;
      rb[p] = (gn < N && k < K) ? *reinterpret_cast<const float4*>(W + (int64_t)gn * ldw + k) : z4;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = (i % F4R) * 4;
      if constexpr (BF16) *reinterpret_cast<bf16x4*>(&As[buf][r][k]) = to_bf16x4(ra[p]);
      else *reinterpret_cast<float4*>(&As[buf][r][k]) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = (i % F4R) * 4;
      if constexpr (BF16) *reinterpret_cast<bf16x4*>(&Bs[buf][r][k]) = to_bf16x4(rb[p]);
      else *reinterpret_cast<float4*>(&Bs[buf][r][k]) = rb[p];
    }
  };
  const int wm = (wv % WM) * 64, wn = (wv / WM) * 64;
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
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = *reinterpret_cast<const bf16x8*>(&As[buf][wm + 16 * i + li][kk + 8 * lq]);
          b[i] = *reinterpret_cast<const bf16x8*>(&Bs[buf][wn + 16 * i + li][kk + 8 * lq]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        f32x4 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = *reinterpret_cast<const f32x4*>(&As[buf][wm + 16 * i + li][kk + 4 * lq]);
          b[i] = *reinterpret_cast<const f32x4*>(&Bs[buf][wn + 16 * i + li][kk + 4 * lq]);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][c], b[j][c], acc[i][j], 0, 0, 0);
      }
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

template <bool BF16, int WM, int BK>
static hipError_t launch_gemm(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K,
                              Epi e, hipStream_t st) {
  const int64_t tiles = (int64_t)((M + 64 * WM - 1) / (64 * WM)) * ((N + 127) / 128);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  gemm_nt_kernel<BF16, WM, BK><<<(unsigned)tiles, 128 * WM, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e);
  return hipGetLastError();
}

// Tile form per dtype: (WM, BK) = (4, 16) fp32, (4, 64) bf16, the best of the four forms
// measured on MI355X (TFLOP/s at M 14000, N 5000, K 5408 / 4096^3; profiles/r2_gemm_bench.txt):
// fp32 73.7 / 75.0 / 89.3 / 73.1 and 84-101; bf16 144-162 (operands converted from fp32 in the
// staging).  One-stage-prefetch kernels whose stage compute is shorter than a loaded memory
// round trip: latency-bound, below hipBLASLt's 141 TF fp32 on the same shapes, which is why the
// fp32 evaluation product is routed to the library (ops/hip_ops.py) and this kernel serves
// --dtype bf16 and graph capture.
hipError_t gemm_nt(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K, Epi e,
                   bool bf16, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if ((K & 3) || (ldx & 3) || (ldw & 3)) return hipErrorInvalidValue;
  if (bf16) return launch_gemm<true, 4, 64>(X, ldx, W, ldw, Y, ldy, M, N, K, e, st);
  return launch_gemm<false, 4, 16>(X, ldx, W, ldw, Y, ldy, M, N, K, e, st);
}

}  // namespace sl
