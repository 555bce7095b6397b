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

#include <algorithm>
#include <type_traits>

namespace sl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// Operand loads are buffer loads with 32-bit byte offsets (operands < 2 GB: gemm_nt splits
// taller X by rows); an out-of-range tile element gets an offset past the buffer and reads as
// 0.  (`cond ? *p : zero` was turned into a load through a select of the global pointer and
// the address of a private zero: flat loads, the staging registers demoted to scratch, and
// every LDS wait also waiting for the prefetch.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gemm_rsrc(const float* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 gemm_ld(__amdgpu_buffer_rsrc_t rs, bool in, int64_t elem) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const int off = in ? (int)(elem * 4) : 0x7ffffff0;
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
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
  const __amdgpu_buffer_rsrc_t rX = gemm_rsrc(X, (int64_t)M * ldx * 4), rW = gemm_rsrc(W, (int64_t)N * ldw * 4);
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = k0 + (i % F4R) * 4, gm = m0 + r;
      ra[p] = gemm_ld(rX, gm < M && k < K, (int64_t)gm * ldx + k);
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = k0 + (i % F4R) * 4, gn = n0 + r;
      rb[p] = gemm_ld(rW, gn < N && k < K, (int64_t)gn * ldw + k);
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
    // next stage's loads in flight during the MFMAs (unconditional: the last stage reloads
    // its own block, unused; a conditional load keeps ra / rb out of registers)
    gload((s + 1 < nk ? s + 1 : s) * BK);
    __builtin_amdgcn_sched_barrier(0);          // the loads go out before the MFMAs
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
    // keep the staging stores (and so the wait for the prefetched data) after this stage's
    // MFMAs: scheduled above them, they expose the whole load latency every stage
    __builtin_amdgcn_sched_barrier(0);
    // the other buffer (its last readers finished before the previous barrier); at the last
    // stage an unused write, kept unconditional so the loads are not sunk below the MFMAs
    sstore(buf ^ 1);
    __syncthreads();
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

// fp32 on the 32 x 32 x 2 MFMA: each wave a 64 x 64 tile as 2 x 2 blocks of 32 x 32
// (4 accumulators of 16 floats).  Lane half h = lane >> 5 holds k = 2 s + h of a step; the
// k order inside a 16-wide stage is permuted so a lane's operands for 8 consecutive steps are
// two contiguous float4s (logical k of step s, half h: 8 h + s), one ds_read_b128 each.
// Split-K (gridDim.y = S > 1, for grids of few tiles): slice z = blockIdx.y covers k in
// [z kc, z kc + kc) and stores its raw partial sums into slab z of P ([S][M][N]); the slabs are
// then reduced with the epilogue applied (linear_epilogue).
// Tail split (tail > 0): this launch covers tiles [tile0, tile0 + tail), gridDim.y = S slices
// each, and slab z of tile j is stored compactly at P[(z tail + j) BM BN] (tail_reduce_kernel
// sums them) -- the last partial round of a large grid spread over S x as many workgroups.
template <int WM, int BK>
__global__ void __launch_bounds__(128 * WM)
gemm_nt_f32x32_kernel(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw,
                      float* __restrict__ Y, int ldy, int M, int N, int K, Epi e, int kc, float* __restrict__ P,
                      int tile0 = 0, int tail = 0) {
  constexpr int BM = 64 * WM, BN = 128, NT = 128 * WM;
  constexpr int LD = BK + 4;
  constexpr int F4R = BK / 4;
  constexpr int APER = BM * F4R / NT, BPER = BN * F4R / NT;
  static_assert(APER * NT == BM * F4R && BPER * NT == BN * F4R, "tile / thread split");
  static_assert(BK % 16 == 0, "16-wide k groups");
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  __shared__ __attribute__((aligned(16))) float As[2][BM][LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tilesM = (M + BM - 1) / BM;
  const int tix = tile0 + (int)blockIdx.x;
  const int tm = tix % tilesM, tn = tix / tilesM;
  const int m0 = tm * BM, n0 = tn * BN;
  float4 ra[APER], rb[BPER];
  const __amdgpu_buffer_rsrc_t rX = gemm_rsrc(X, (int64_t)M * ldx * 4), rW = gemm_rsrc(W, (int64_t)N * ldw * 4);
  const int kb = (int)blockIdx.y * kc, ke = min(K, kb + kc);
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = k0 + (i % F4R) * 4, gm = m0 + r;
      ra[p] = gemm_ld(rX, gm < M && k < ke, (int64_t)gm * ldx + k);
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = k0 + (i % F4R) * 4, gn = n0 + r;
      rb[p] = gemm_ld(rW, gn < N && k < ke, (int64_t)gn * ldw + k);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = (i % F4R) * 4;
      *reinterpret_cast<float4*>(&As[buf][r][k]) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = i / F4R, k = (i % F4R) * 4;
      *reinterpret_cast<float4*>(&Bs[buf][r][k]) = rb[p];
    }
  };
  const int wm = (wv % WM) * 64, wn = (wv / WM) * 64;
  const int lr = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (ke - kb + BK - 1) / BK;
  gload(kb);
  sstore(0);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    gload(kb + (s + 1 < nk ? s + 1 : s) * BK);
    __builtin_amdgcn_sched_barrier(0);          // the loads go out before the MFMAs
    // raised issue priority while this wave feeds its MFMAs: +1.7-2.7 % at 14000 x 5000 x 5408,
    // 14000 x 1000 x 5000 and 4096^3 (profiles/r4u_gemm_setprio_ab.txt)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      f32x4 a[2][2], b[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          a[i][q] = *reinterpret_cast<const f32x4*>(&As[buf][wm + 32 * i + lr][kk + 8 * h + 4 * q]);
          b[i][q] = *reinterpret_cast<const f32x4*>(&Bs[buf][wn + 32 * i + lr][kk + 8 * h + 4 * q]);
        }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q][c], b[j][q][c], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    sstore(buf ^ 1);
    __syncthreads();
  }
  // C / D: lane l of block (i, j), register r: row 32 i + (r & 3) + 8 (r >> 2) + 4 h, column 32 j + l & 31
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 32 * j + lr;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= M) continue;
        if (tail > 0)
          P[(((int64_t)blockIdx.y * tail + blockIdx.x) * BM + (m - m0)) * BN + (n - n0)] = acc[i][j][r];
        else if (P)
          P[((int64_t)blockIdx.y * M + m) * N + n] = acc[i][j][r];
        else
          Y[(int64_t)m * ldy + n] = apply_epi(e, acc[i][j][r], m, n);
      }
    }
}

// Y of the tail tiles = epi(sum of their S compact slabs, in slice order)
template <int BM>
__global__ void __launch_bounds__(256) tail_reduce_kernel(const float* __restrict__ P, int S, int tail, int tile0,
                                                          float* __restrict__ Y, int ldy, int M, int N, Epi e) {
  constexpr int BN = 128;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)tail * BM * BN) return;
  const int j = (int)(t / (BM * BN)), rc = (int)(t - (int64_t)j * BM * BN);
  const int tilesM = (M + BM - 1) / BM, tix = tile0 + j;
  const int m = (tix % tilesM) * BM + rc / BN, n = (tix / tilesM) * BN + rc % BN;
  if (m >= M || n >= N) return;
  float v = P[t];
  for (int z = 1; z < S; ++z) v += P[(int64_t)z * tail * BM * BN + t];
  Y[(int64_t)m * ldy + n] = apply_epi(e, v, m, n);
}

// NN layout for the data gradient of many rows: dX[M, K] = mask(dZ[M, R] . W[R, K]) (W as
// stored, [out features][in features]; reference: the backward of nn.Linear through
// split_nn.py:156's --batch_size rows, data_entities_vanilla.py:231).  Same 32 x 32 x 2 fp32
// MFMA tiling as gemm_nt_f32x32_kernel (BM x 128 output tile, 16-deep reduction stages,
// double-buffered LDS, next stage's loads before this stage's MFMAs).  A (= dZ) is staged as
// in the NT form; B (= W) is read along its rows (coalesced float4 along the output columns)
// and kept in LDS as [reduction][column] (pitch 132: the two lane halves' rows land 32 banks
// apart), each MFMA's B operand one conflict-free scalar read per lane (the float4-per-k
// reads of the NT form would need a transposed, 8-way bank-conflicted staging store).
// Epilogue: the previous layer's ReLU / dropout mask (hprev > 0 ? v scale : 0) fused into the
// store; split over the reduction (gridDim.y = S > 1) stores raw slabs to P, reduced and
// masked by dgrad_reduce.
template <int WM>
__global__ void __launch_bounds__(128 * WM)
gemm_nn_f32x32_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb,
                      float* __restrict__ Y, int ldy, int M, int N, int R, const float* __restrict__ hprev, int ldh,
                      float scale, int kc, float* __restrict__ P) {
  constexpr int BM = 64 * WM, BN = 128, NT = 128 * WM, BK = 16;
  constexpr int LDA = BK + 4, LDB = BN + 4;
  constexpr int F4A = BK / 4, F4B = BN / 4;
  constexpr int APER = BM * F4A / NT, BPER = BK * F4B / NT;
  static_assert(APER * NT == BM * F4A && BPER * NT == BK * F4B, "tile / thread split");
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  __shared__ __attribute__((aligned(16))) float As[2][BM][LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tilesM = (M + BM - 1) / BM;
  const int tm = blockIdx.x % tilesM, tn = blockIdx.x / tilesM;
  const int m0 = tm * BM, n0 = tn * BN;
  float4 ra[APER], rb[BPER];
  const __amdgpu_buffer_rsrc_t rA = gemm_rsrc(A, (int64_t)M * lda * 4), rB = gemm_rsrc(B, (int64_t)R * ldb * 4);
  const int kb = (int)blockIdx.y * kc, ke = min(R, kb + kc);
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4A, k = k0 + (i % F4A) * 4, gm = m0 + r;
      ra[p] = gemm_ld(rA, gm < M && k < ke, (int64_t)gm * lda + k);
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = k0 + i / F4B, c = n0 + (i % F4B) * 4;
      rb[p] = gemm_ld(rB, r < ke && c < N, (int64_t)r * ldb + c);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < APER; ++p) {
      const int i = tid + p * NT, r = i / F4A, k = (i % F4A) * 4;
      *reinterpret_cast<float4*>(&As[buf][r][k]) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BPER; ++p) {
      const int i = tid + p * NT, r = i / F4B, c = (i % F4B) * 4;
      *reinterpret_cast<float4*>(&Bs[buf][r][c]) = rb[p];
    }
  };
  const int wm = (wv % WM) * 64, wn = (wv / WM) * 64;
  const int lr = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (ke - kb + BK - 1) / BK;
  gload(kb);
  sstore(0);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    gload(kb + (s + 1 < nk ? s + 1 : s) * BK);
    __builtin_amdgcn_sched_barrier(0);          // the loads go out before the MFMAs
    __builtin_amdgcn_s_setprio(1);             // as gemm_nt_f32x32_kernel
    // step (q, c) of lane half h reduces logical k = 8 h + 4 q + c (the NT form's order)
    f32x4 a[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q) a[i][q] = *reinterpret_cast<const f32x4*>(&As[buf][wm + 32 * i + lr][8 * h + 4 * q]);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = 8 * h + 4 * q + c;
        const float b0 = Bs[buf][k][wn + lr], b1 = Bs[buf][k][wn + 32 + lr];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q][c], b0, acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q][c], b1, acc[i][1], 0, 0, 0);
        }
      }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 32 * j + lr;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= M) continue;
        const float v = acc[i][j][r];
        if (P) {
          P[((int64_t)blockIdx.y * M + m) * N + n] = v;
        } else {
          Y[(int64_t)m * ldy + n] = hprev ? (hprev[(int64_t)m * ldh + n] > 0.f ? v * scale : 0.f) : v;
        }
      }
    }
}

hipError_t dgrad_reduce(const float* P, int S, int64_t slab, const float* hprev, int ldh, float scale, float* out,
                        int ldo, int M, int K, hipStream_t st);

// dX[M, K] = mask(dZ[M, R] . W[R, K]): 256 x 128 tiles when they fill the chip, else 128 x 128
// tiles split over the reduction (the choice below).
hipError_t gemm_nn_dgrad(const float* dZ, int ldz, const float* W, int ldw, const float* hprev, int ldh, float scale,
                         float* dX, int ldx, int M, int R, int K, float* ws, int64_t ws_elems, hipStream_t st) {
  if (M <= 0 || K <= 0) return hipSuccess;
  if ((R & 3) || (K & 3) || (ldz & 3) || (ldw & 3)) return hipErrorInvalidValue;
  constexpr int64_t kMax = 0x7fff0000;
  if ((int64_t)M * ldz * 4 > kMax || (int64_t)R * ldw * 4 > kMax) return hipErrorInvalidValue;
  const int64_t t4 = (int64_t)((M + 255) / 256) * ((K + 127) / 128);
  if (t4 >= 384 && g_nn_wm != 2) {
    gemm_nn_f32x32_kernel<4><<<(unsigned)t4, 512, 0, st>>>(dZ, ldz, W, ldw, dX, ldx, M, K, R, hprev, ldh, scale, R,
                                                          nullptr);
    return hipGetLastError();
  }
  if (g_nn_wm == 4 && g_nn_splits > 0) {   // A/B: the 256 x 128 form split over the reduction
    const int S4 = std::max(1, std::min<int>(g_nn_splits, (int)std::min<int64_t>(64, ws ? ws_elems / ((int64_t)M * K) : 0)));
    const int kc4 = S4 > 1 ? ((R + S4 - 1) / S4 + 15) / 16 * 16 : R;
    gemm_nn_f32x32_kernel<4><<<dim3((unsigned)t4, S4), 512, 0, st>>>(dZ, ldz, W, ldw, dX, ldx, M, K, R, hprev, ldh,
                                                                    scale, kc4, S4 > 1 ? ws : nullptr);
    if (S4 > 1) return dgrad_reduce(ws, S4, (int64_t)M * K, hprev, ldh, scale, dX, ldx, M, K, st);
    return hipGetLastError();
  }
  const int64_t t2 = (int64_t)((M + 127) / 128) * ((K + 127) / 128);
  if (t2 > 0x7fffffff) return hipErrorInvalidValue;
  int S = 1;
  if (ws == nullptr) ws_elems = 0;
  // The split over the reduction (profiles/r6_gemm/nn_sweep_form2.txt, every S 1-32 at the eval /
  // large-batch shapes against hipBLASLt): a long reduction takes 8 slices (workgroups are then
  // short, so the last one to finish trails the grid by little; the slab reduce costs ~6 %), a
  // short one ~640 / tiles slices of >= 128 (beyond that the slab reduce and the fixed costs of
  // a workgroup win).  M = 200: 60 -> 82 % of hipBLASLt at R = 5000, 55 -> 72 % at R = 1000;
  // M = 1000: 72 -> 97 %, 76 -> 75 %.
  const int64_t smax = ws_elems / std::max<int64_t>(1, (int64_t)M * K);
  if (R >= 2048) S = 8;
  else S = (int)std::min<int64_t>(6, std::max<int64_t>(1, (640 + t2 / 2) / std::max<int64_t>(1, t2)));
  while (S > 1 && (R / S < (t2 < 32 ? 64 : 128) || S > smax)) --S;
  if (g_nn_splits > 0) S = std::max(1, std::min<int>(g_nn_splits, (int)std::min<int64_t>(64, ws_elems / ((int64_t)M * K))));
  const int kc = S > 1 ? ((R + S - 1) / S + 15) / 16 * 16 : R;
  gemm_nn_f32x32_kernel<2><<<dim3((unsigned)t2, S), 256, 0, st>>>(dZ, ldz, W, ldw, dX, ldx, M, K, R, hprev, ldh,
                                                                 scale, kc, S > 1 ? ws : nullptr);
  if (S > 1) return dgrad_reduce(ws, S, (int64_t)M * K, hprev, ldh, scale, dX, ldx, M, K, st);
  return hipGetLastError();
}

hipError_t linear_epilogue(const float* P, int ldp, float* Y, int ldy, int M, int N, Epi e, int S, int64_t slab,
                           hipStream_t st);

// S > 1: split-K over S slices into ws ([S][M][N], >= S M N floats), then one reduce +
// epilogue launch.
template <int WM, int BK>
static hipError_t launch_gemm_f32x32(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N,
                                     int K, Epi e, int S, float* ws, hipStream_t st) {
  const int64_t tiles = (int64_t)((M + 64 * WM - 1) / (64 * WM)) * ((N + 127) / 128);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  const int kc = S > 1 ? ((K + S - 1) / S + BK - 1) / BK * BK : K;
  gemm_nt_f32x32_kernel<WM, BK><<<dim3((unsigned)tiles, S), 128 * WM, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e,
                                                                             kc, S > 1 ? ws : nullptr);
  if (S > 1) return linear_epilogue(ws, N, Y, ldy, M, N, e, S, (int64_t)M * N, st);
  return hipGetLastError();
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
static hipError_t gemm_nt_rows(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N,
                               int K, Epi e, bool bf16, float* ws, int64_t ws_elems, hipStream_t st);

// compute units of the current device (cached per device)
static int gemm_cus() {
  static int cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

hipError_t gemm_nt(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K, Epi e,
                   bool bf16, float* ws, int64_t ws_elems, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if ((K & 3) || (ldx & 3) || (ldw & 3)) return hipErrorInvalidValue;
  constexpr int64_t kMax = 0x7fff0000;            // buffer-load byte offsets (gemm_ld)
  if ((int64_t)N * ldw * 4 > kMax || (int64_t)ldx * 4 * 256 > kMax) return hipErrorInvalidValue;
  const int rows = (int)std::min<int64_t>(M, kMax / ((int64_t)ldx * 4) / 256 * 256);
  // the dropout hash takes the row index: a chunked product would restart it (inference only)
  if (rows < M && e.thresh) return hipErrorInvalidValue;
  for (int m = 0; m < M; m += rows) {
    const hipError_t r = gemm_nt_rows(X + (int64_t)m * ldx, ldx, W, ldw, Y + (int64_t)m * ldy, ldy,
                                      std::min(rows, M - m), N, K, e, bf16, ws, ws_elems, st);
    if (r != hipSuccess) return r;
  }
  return hipSuccess;
}

static hipError_t gemm_nt_rows(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N,
                               int K, Epi e, bool bf16, float* ws, int64_t ws_elems, hipStream_t st) {
  if (!ws) ws_elems = 0;
  if (bf16) return launch_gemm<true, 4, 64>(X, ldx, W, ldw, Y, ldy, M, N, K, e, st);
  switch (g_variant[10]) {   // A/B of the fp32 forms (scripts/gemm_bench.py)
    case 1: return launch_gemm_f32x32<2, 16>(X, ldx, W, ldw, Y, ldy, M, N, K, e, 1, nullptr, st);
    case 2: return launch_gemm_f32x32<4, 16>(X, ldx, W, ldw, Y, ldy, M, N, K, e, 1, nullptr, st);
    case 3: return launch_gemm_f32x32<2, 32>(X, ldx, W, ldw, Y, ldy, M, N, K, e, 1, nullptr, st);
    case 4: return launch_gemm_f32x32<4, 32>(X, ldx, W, ldw, Y, ldy, M, N, K, e, 1, nullptr, st);
    case 5: return launch_gemm<false, 4, 16>(X, ldx, W, ldw, Y, ldy, M, N, K, e, st);
    default: break;
  }
  // fp32: the 32 x 32 x 2 form.  256 x 128 tiles when they fill the chip (>= 1.5 per CU:
  // M 14000, N 1000 measured 108.8 vs 104.4 TF/s against 128 x 128 tiles), else 128 x 128
  // tiles, split over K until ~2 workgroups per CU (slices >= 512 deep, >= 256 when fewer
  // tiles than CUs: M 14000, N 100, K 1000 ran 110 workgroups; <= 8 slices; a grid of a few
  // tiles, whose time is its stage count times a loaded round trip, down to 64 deep:
  // M 1000, N 100, K 1000 is 8 tiles)
  const int64_t t4 = (int64_t)((M + 255) / 256) * ((N + 127) / 128);
  if (t4 >= 384) {
    // whole rounds of the resident slots (2 workgroups per CU) as full-K tiles; a last round
    // under 3/4 full is instead split over K into up to S x its tiles (tail_reduce_kernel sums
    // them): M 14000, N 5000 is 4 rounds of 512 plus 152 tiles
    const int64_t slots = 2LL * gemm_cus();
    const int64_t rem = t4 % slots, full = t4 - rem;
    int S = 1;
    if (full > 0 && rem > 0 && 4 * rem < 3 * slots) {
      S = (int)std::min<int64_t>(8, slots / rem);
      while (S > 1 && (K / S < 512 || (int64_t)S * rem * 256 * 128 > ws_elems)) --S;
    }
    // (a row-band tile order for L2 reuse within an XCD measured the same: 127.4 vs 127.2 TF at
    // 14000 x 5000 x 5408, profiles/r4h_gemm_tile_order_ab.txt)
    if (S == 1) return launch_gemm_f32x32<4, 16>(X, ldx, W, ldw, Y, ldy, M, N, K, e, 1, nullptr, st);
    gemm_nt_f32x32_kernel<4, 16><<<(unsigned)full, 512, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, K, nullptr);
    const int kc = ((K + S - 1) / S + 15) / 16 * 16;
    gemm_nt_f32x32_kernel<4, 16><<<dim3((unsigned)rem, S), 512, 0, st>>>(X, ldx, W, ldw, Y, ldy, M, N, K, e, kc, ws,
                                                                        (int)full, (int)rem);
    const int64_t tot = rem * 256 * 128;
    tail_reduce_kernel<256><<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(ws, S, (int)rem, (int)full, Y, ldy, M, N,
                                                                          e);
    return hipGetLastError();
  }
  const int64_t t2 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  const int kmin = t2 < 32 ? 64 : t2 < 256 ? 256 : 512;
  int S = 1;
  // up to 8 slices, or one workgroup per CU for a grid of under 32 tiles (M = 200, N = 1000, K =
  // 5000: 16 tiles x 16 slices, 48 -> 74 % of hipBLASLt; profiles/r6_gemm/nt_sweep_wide.txt)
  const int smax2 = t2 < 32 ? std::max<int>(8, (int)(256 / std::max<int64_t>(1, t2))) : 8;
  while (S < smax2 && t2 * S * 2 <= 640 && K / (S * 2) >= kmin && (int64_t)S * 2 * M * N <= ws_elems) S *= 2;
  // a long reduction over >= 80 tiles: 6 slices (profiles/r6_gemm/nt_sweep.txt, against
  // hipBLASLt: M = 200, N = 5000, K = 5408 78 -> 90 %, M = 1000 81 -> 89 %)
  if (t2 >= 80 && K >= 4096 && (int64_t)6 * M * N <= ws_elems) S = 6;
  if (g_nt_splits > 0) S = std::max(1, std::min<int>(g_nt_splits, (int)std::min<int64_t>(64, ws_elems / ((int64_t)M * N))));
  return launch_gemm_f32x32<2, 16>(X, ldx, W, ldw, Y, ldy, M, N, K, e, S, ws, st);
}

}  // namespace sl
