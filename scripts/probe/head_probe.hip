// Standalone timing probe of Bob's server head kernels (fused.hip head_fwd / head_bwd) at the
// server-step shape (M 16, fc2 N 1000, C 100, 16 fc2 split-K slabs): back-to-back launches
// (L2-hot) and launches behind a 512 MB memset (cold), against an empty kernel, plus
// dissected forms of head_fwd (slab phase only / logits phase only).  Not part of the
// package; built by scripts/probe/build.sh, run on the GPU box.
#include "../../splitlearning_amd/csrc/linear.hip"
#include "../../splitlearning_amd/csrc/fused.hip"
#include "../../splitlearning_amd/csrc/gemm.hip"

#include <cstdio>
#include <vector>

using namespace sl;

static hipStream_t g_probe_stream = 0;

// head_fwd_v0_kernel (the round-1 form, kept here for the A/B): workgroup (m, q) reduces fc2's split-K slabs for its column slice of row
// m, applies fc2's epilogue (-> h2) and writes the slice's partial fc3 logits plog[q][m][:].
// Every load of a phase is issued before the first is consumed (one memory round trip per
// phase): at B = 16 this op is pure latency.
__global__ void __launch_bounds__(256)
head_fwd_v0_kernel(const float* __restrict__ P2, int S2, int64_t slab2, Epi e2, const float* __restrict__ W3,
                int ldw3, float* __restrict__ h2, float* __restrict__ plog, int M, int N2, int C, int bf) {
  __shared__ f32x4 part[8][HS];
  __shared__ f32x4 hs[HS];
  const int m = blockIdx.x, q = blockIdx.y, Q = gridDim.y, tid = threadIdx.x;
  int qa, qb;
  head_slice(N2 >> 2, Q, q, qa, qb);
  const int ncol = qb - qa;
  const int lane = tid & 63, wv = tid >> 6, half = lane >> 5, c = lane & 31;
  constexpr int JU = 13;
  // W3 loads of the first output group do not depend on anything: issue them first so
  // they overlap the slab reduction (one memory round trip for the whole kernel at C <= 104)
  f32x4 w[JU];
  auto load_w = [&](int j0) {
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * (j0 + j) + 2 * wv + half;
      w[j] = (o < C && c < ncol) ? *reinterpret_cast<const f32x4*>(W3 + (int64_t)o * ldw3 + 4 * (qa + c))
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  load_w(0);
  // 1. slab reduction: 32 columns x 8 slab groups
  {
    const int c = tid & (HS - 1), sg = tid >> 5;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (c < ncol) {
      const f32x4* src = reinterpret_cast<const f32x4*>(P2 + (int64_t)m * N2) + qa + c;
#pragma unroll 4
      for (int s = sg; s < S2; s += 8) v += src[s * (slab2 >> 2)];
    }
    part[sg][c] = v;
  }
  __syncthreads();
  if (tid < HS) {
    f32x4 v = part[0][tid];
#pragma unroll
    for (int g = 1; g < 8; ++g) v += part[g][tid];
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    if (tid < ncol) {
      const int col = 4 * (qa + tid);
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = apply_epi(e2, v[i], m, col + i);
      reinterpret_cast<f32x4*>(h2 + (int64_t)m * N2)[qa + tid] = o;
    }
    hs[tid] = o;
  }
  __syncthreads();
  // 2. partial logits: half-waves (32 lanes = the slice's columns) per output, 8 outputs
  //    per wave instruction group; JU outputs' loads in flight per lane
  const f32x4 h = bf ? bfr4(hs[c]) : hs[c];
  for (int j0 = 0; j0 * 8 < C; j0 += JU) {
    if (j0) load_w(j0);
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * (j0 + j) + 2 * wv + half;
      const f32x4 wj = bf ? bfr4(w[j]) : w[j];
      float d = wj[0] * h[0] + wj[1] * h[1] + wj[2] * h[2] + wj[3] * h[3];
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) d += __shfl_xor(d, off);
      if (c == 0 && o < C) plog[((int64_t)q * M + m) * C + o] = d;
    }
  }
}

// head_bwd_v0_kernel (the round-1 form, kept here for the A/B): workgroup (m, q) sums row m's partial logits (+ b3), softmax-CE (loss and
// dlogits written by q == 0), then dz2 = (dlogits . W3) * dscale * [h2 > 0] for its slice.
__global__ void __launch_bounds__(256)
head_bwd_v0_kernel(const float* __restrict__ plog, const float* __restrict__ b3, const float* __restrict__ W3,
                int ldw3, const int64_t* __restrict__ y, int64_t ignore, float scale, float dscale,
                const float* __restrict__ h2, float* __restrict__ dlog, float* __restrict__ dz2,
                float* __restrict__ loss_rows, int M, int N2, int C, int bf, int Qp) {
  // Qp: number of partial-logit slabs in plog (head_fwd: one per column slice = gridDim.y;
  // fc2_head_fwd: one per 8-column tile)
  extern __shared__ float lg[];   // C
  __shared__ f32x4 part[8][HS];
  const int m = blockIdx.x, q = blockIdx.y, Q = gridDim.y, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  int qa, qb;
  head_slice(N2 >> 2, Q, q, qa, qb);
  const int ncol = qb - qa;
  const int c = tid & (HS - 1), g = tid >> 5;
  constexpr int JU = 13;
  // independent loads first: this slice's W3 columns (first output group) and h2 mask
  f32x4 w[JU];
  auto load_w = [&](int j0) {
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * (j0 + j) + g;
      w[j] = (o < C && c < ncol) ? *reinterpret_cast<const f32x4*>(W3 + (int64_t)o * ldw3 + 4 * (qa + c))
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  load_w(0);
  f32x4 hh = {0.f, 0.f, 0.f, 0.f};
  if (tid < ncol) hh = reinterpret_cast<const f32x4*>(h2 + (int64_t)m * N2)[qa + tid];
  for (int o = tid; o < C; o += 256) {
    float v = b3 ? b3[o] : 0.f;
#pragma unroll 8
    for (int s = 0; s < Qp; ++s) v += plog[((int64_t)s * M + m) * C + o];
    lg[o] = v;
  }
  __syncthreads();
  const int64_t lab = y[m];
  if (wv == 0) {
    if (lab == ignore) {
      for (int c = lane; c < C; c += 64) lg[c] = 0.f;
      if (lane == 0 && q == 0) loss_rows[m] = 0.f;
    } else {
      float mx = -INFINITY;
      for (int c = lane; c < C; c += 64) mx = fmaxf(mx, lg[c]);
      for (int o_ = 32; o_ > 0; o_ >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o_, 64));
      float se = 0.f;
      for (int c = lane; c < C; c += 64) se += expf(lg[c] - mx);
      for (int o_ = 32; o_ > 0; o_ >>= 1) se += __shfl_xor(se, o_, 64);
      if (lane == 0 && q == 0) loss_rows[m] = mx + logf(se) - lg[lab];
      const float inv = 1.f / se;
      for (int c = lane; c < C; c += 64) {
        float p = expf(lg[c] - mx) * inv;
        if (c == lab) p -= 1.f;
        lg[c] = p * scale;
      }
    }
  }
  __syncthreads();
  if (q == 0)
    for (int cc = tid; cc < C; cc += 256) dlog[(int64_t)m * C + cc] = lg[cc];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 * 8 < C; j0 += JU) {
    if (j0) load_w(j0);
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * (j0 + j) + g;
      const float l = o < C ? lg[o] : 0.f;
      acc += bf ? bfr(l) * bfr4(w[j]) : l * w[j];
    }
  }
  part[g][c] = acc;
  __syncthreads();
  if (tid < ncol) {
    f32x4 v = part[0][tid];
#pragma unroll
    for (int gg = 1; gg < 8; ++gg) v += part[gg][tid];
    f32x4 out;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = hh[i] > 0.f ? v[i] * dscale : 0.f;
    reinterpret_cast<f32x4*>(dz2 + (int64_t)m * N2)[qa + tid] = out;
  }
}


static int head3m_slices(int N2) { return max(1, (N2 / 4 + 15) / 16); }

// head_fwd_mfma_kernel (measured here; not in the package): workgroup q owns a slice of <= 64 fc2 columns
// for ALL M <= 16 rows.  Its fc3 W3 slice (the first loads issued: 2 output tiles x 4 float4
// per lane) is read once per slice instead of once per (row, slice), and the partial logits
// plog[q][m][o] come out of exact-fp32 MFMAs (A = h2 slice from LDS, B = W3 slice) instead
// of per-row dot products reduced by 5-step lane shuffles (the logits phase of head_fwd was
// 2.6 us above an empty launch in a graph-replay probe, scripts/probe/head_probe.hip).
// grid Q = ceil(N2 / 64), 256 threads; C <= 128.
__global__ void __launch_bounds__(256)
head_fwd_mfma_kernel(const float* __restrict__ P2, int S2, int64_t slab2, Epi e2, const float* __restrict__ W3,
                     int ldw3, float* __restrict__ h2, float* __restrict__ plog, int M, int N2, int C, int bf) {
  __shared__ __attribute__((aligned(16))) float hs[16][68];
  const int q = blockIdx.x, Q = gridDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int qa, qb;
  head_slice(N2 >> 2, Q, q, qa, qb);
  const int ncol = 4 * (qb - qa), c0 = 4 * qa;    // this slice's columns [c0, c0 + ncol), ncol <= 64
  const int li = lane & 15, lq = lane >> 4;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  // W3 slice, MFMA B layout: wave wv owns output tiles wv and wv + 4 (16 outputs each); lane
  // (li, lq) holds W3[16 t + li][c0 + 16 g + 4 lq + 0..3] for k-group g
  f32x4 wb[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int o = 16 * (wv + 4 * t) + li;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = 16 * g + 4 * lq;
      wb[t][g] = (o < C && col < ncol) ? *reinterpret_cast<const f32x4*>(W3 + (int64_t)o * ldw3 + c0 + col) : z;
    }
  }
  // fc2's split-K slabs for (row m, float4 column f), every slab load in flight at once
  const int m = tid >> 4, f = tid & 15;
  const bool own = m < M && 4 * f < ncol;
  f32x4 v = z;
  if (own) {
    const f32x4* src = reinterpret_cast<const f32x4*>(P2 + (int64_t)m * N2 + c0) + f;
    f32x4 r[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) r[s] = s < S2 ? src[s * (slab2 >> 2)] : z;
#pragma unroll
    for (int s = 0; s < 16; ++s) v += r[s];
    for (int s = 16; s < S2; ++s) v += src[s * (slab2 >> 2)];
  }
  f32x4 o4 = z;
  if (own) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o4[i] = apply_epi(e2, v[i], m, c0 + 4 * f + i);
    reinterpret_cast<f32x4*>(h2 + (int64_t)m * N2 + c0)[f] = o4;
  }
  *reinterpret_cast<f32x4*>(&hs[m][4 * f]) = bf ? bfr4(o4) : o4;
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ot = wv + 4 * t;
    if (16 * ot >= C) break;                        // wave-uniform
    f32x4 acc = z;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&hs[li][16 * g + 4 * lq]);
      const f32x4 w = bf ? bfr4(wb[t][g]) : wb[t][g];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], w[j], acc, 0, 0, 0);
    }
    // lane (li = output column, lq): rows 4 lq + r
    const int o = 16 * ot + li;
    if (o < C) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = 4 * lq + r;
        if (mm < M) plog[((int64_t)q * M + mm) * C + o] = acc[r];
      }
    }
  }
}

// head_bwd_mfma_kernel (measured here; pairs with head_fwd_mfma_kernel): workgroup q owns a
// slice of <= 64 fc2 columns for ALL M <= 16 rows.  Every workgroup sums the Qp partial
// logit slabs of all rows (one round trip: <= 32 float4 loads per thread) and runs the
// softmax-CE of all rows redundantly (16-lane groups, one row each, in-row reductions over
// 16 lanes), so no workgroup waits on another; q == 0 writes dlogits and the losses.  Then
// dz2[:, slice] = (dlogits . W3[:, slice]) * dscale * [h2 > 0] through exact-fp32 MFMAs
// (A = dlogits from LDS, B = W3 column tile; wave w owns the slice's 16-column tile w), with
// the W3 and h2 loads issued first.  grid Q = ceil(N2 / 64), 256 threads; C <= 128.
__global__ void __launch_bounds__(256)
head_bwd_mfma_kernel(const float* __restrict__ plog, const float* __restrict__ b3, const float* __restrict__ W3,
                     int ldw3, const int64_t* __restrict__ y, int64_t ignore, float scale, float dscale,
                     const float* __restrict__ h2, float* __restrict__ dlog, float* __restrict__ dz2,
                     float* __restrict__ loss_rows, int M, int N2, int C, int bf, int Qp) {
  __shared__ __attribute__((aligned(16))) float lg[16][132];
  const int q = blockIdx.x, Q = gridDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int qa, qb;
  head_slice(N2 >> 2, Q, q, qa, qb);
  const int ncol = 4 * (qb - qa), c0 = 4 * qa;
  const int li = lane & 15, lq = lane >> 4;
  // independent loads first: W3[o][c0 + 16 wv + li] for o = 4 s + lq (MFMA B layout, k = o)
  // and the h2 mask of this lane's output column
  const int col = 16 * wv + li;
  const bool vcol = col < ncol;
  float wb[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    const int o = 4 * s + lq;
    wb[s] = (vcol && o < C) ? W3[(int64_t)o * ldw3 + c0 + col] : 0.f;
  }
  float hm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = 4 * lq + r;
    hm[r] = (vcol && m < M) ? h2[(int64_t)m * N2 + c0 + col] : 0.f;
  }
  // logits: thread -> (row m = tid >> 4, float4 columns f = tid & 15, + 16, ...) over C/4
  {
    const int m = tid >> 4, f0 = tid & 15;
    const int C4 = C >> 2;                         // C % 4 == 0 here (host check)
    if (m < M) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int f = f0 + 16 * i;
        if (f < C4) {
          f32x4 r[16];
          const f32x4* src = reinterpret_cast<const f32x4*>(plog + (int64_t)m * C) + f;
          const int64_t st4 = (int64_t)M * C >> 2;
#pragma unroll
          for (int s = 0; s < 16; ++s) r[s] = s < Qp ? src[s * st4] : f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4 v = b3 ? reinterpret_cast<const f32x4*>(b3)[f] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 16; ++s) v += r[s];
          for (int s = 16; s < Qp; ++s) v += src[s * st4];
          *reinterpret_cast<f32x4*>(&lg[m][4 * f]) = v;
        }
      }
    }
  }
  __syncthreads();
  // softmax-CE: 16-lane group (wave wv, lq) owns row m = 4 wv + lq; lane li takes o = li + 16 i
  {
    const int m = 4 * wv + lq;
    if (m < M) {
      const int64_t lab = y[m];
      if (lab == ignore) {
        for (int o = li; o < C; o += 16) lg[m][o] = 0.f;
        if (li == 0 && q == 0) loss_rows[m] = 0.f;
      } else {
        float mx = -INFINITY;
        for (int o = li; o < C; o += 16) mx = fmaxf(mx, lg[m][o]);
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 16));
        float se = 0.f;
        for (int o = li; o < C; o += 16) se += expf(lg[m][o] - mx);
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) se += __shfl_xor(se, off, 16);
        if (li == 0 && q == 0) loss_rows[m] = mx + logf(se) - lg[m][lab];
        const float inv = 1.f / se;
        for (int o = li; o < C; o += 16) {
          float p = expf(lg[m][o] - mx) * inv;
          if (o == lab) p -= 1.f;
          lg[m][o] = p * scale;
        }
      }
    } else {
      for (int o = li; o < C; o += 16) lg[m][o] = 0.f;
    }
    // lanes past C in the 32 k-steps of the MFMA read lg[m][C..127]: zero them
    for (int o = C + li; o < 128; o += 16) lg[m][o] = 0.f;
  }
  __syncthreads();
  if (q == 0)
    for (int i = tid; i < M * C; i += 256) dlog[i] = lg[i / C][i % C];
  // dz2 tile: D[m][col] = sum_o dlog[m][o] W3[o][col]; A lane (li = m, lq): dlog[li][4 s + lq]
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    if (4 * s >= C) break;
    const float a = lg[li][4 * s + lq];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bf ? bfr(a) : a, bf ? bfr(wb[s]) : wb[s], acc, 0, 0, 0);
  }
  if (vcol) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * lq + r;
      if (m < M) dz2[(int64_t)m * N2 + c0 + col] = hm[r] > 0.f ? acc[r] * dscale : 0.f;
    }
  }
}


__global__ void empty_kernel(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345.f) p[1] = 1.f;
}

// head_fwd dissected: PH = 1 slab phase only, 2 logits phase only (h = hs from LDS zeros)
template <int PH>
__global__ void __launch_bounds__(256)
head_fwd_part(const float* __restrict__ P2, int S2, int64_t slab2, Epi e2, const float* __restrict__ W3, int ldw3,
              float* __restrict__ h2, float* __restrict__ plog, int M, int N2, int C) {
  __shared__ f32x4 part[8][HS];
  __shared__ f32x4 hs[HS];
  const int m = blockIdx.x, q = blockIdx.y, Q = gridDim.y, tid = threadIdx.x;
  int qa, qb;
  head_slice(N2 >> 2, Q, q, qa, qb);
  const int ncol = qb - qa;
  const int lane = tid & 63, wv = tid >> 6, half = lane >> 5, c = lane & 31;
  constexpr int JU = 13;
  f32x4 w[JU];
  if (PH == 2) {
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * j + 2 * wv + half;
      w[j] = (o < C && c < ncol) ? *reinterpret_cast<const f32x4*>(W3 + (int64_t)o * ldw3 + 4 * (qa + c))
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (tid < HS) hs[tid] = f32x4{1.f, 1.f, 1.f, 1.f};
    __syncthreads();
    const f32x4 h = hs[c];
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * j + 2 * wv + half;
      float d = w[j][0] * h[0] + w[j][1] * h[1] + w[j][2] * h[2] + w[j][3] * h[3];
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) d += __shfl_xor(d, off);
      if (c == 0 && o < C) plog[((int64_t)q * M + m) * C + o] = d;
    }
  } else {
    const int cc = tid & (HS - 1), sg = tid >> 5;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (cc < ncol) {
      const f32x4* src = reinterpret_cast<const f32x4*>(P2 + (int64_t)m * N2) + qa + cc;
#pragma unroll 4
      for (int s = sg; s < S2; s += 8) v += src[s * (slab2 >> 2)];
    }
    part[sg][cc] = v;
    __syncthreads();
    if (tid < HS) {
      f32x4 vv = part[0][tid];
#pragma unroll
      for (int g = 1; g < 8; ++g) vv += part[g][tid];
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
      if (tid < ncol) {
        const int col = 4 * (qa + tid);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = apply_epi(e2, vv[i], m, col + i);
        reinterpret_cast<f32x4*>(h2 + (int64_t)m * N2)[qa + tid] = o;
      }
    }
  }
}


// head_bwd dissected: SKIP bit 1 = no plog reduction (logits = b3), 2 = no softmax (dlogits =
// logits), 4 = no dz2 phase (W3 loads and FMAs dropped, zeros stored)
template <int SKIP>
__global__ void __launch_bounds__(256)
head_bwd_part(const float* __restrict__ plog, const float* __restrict__ b3, const float* __restrict__ W3, int ldw3,
              const int64_t* __restrict__ y, int64_t ignore, float scale, float dscale, const float* __restrict__ h2,
              float* __restrict__ dlog, float* __restrict__ dz2, float* __restrict__ loss_rows, int M, int N2, int C,
              int Qp) {
  extern __shared__ float lg[];
  __shared__ f32x4 part[8][HS];
  const int m = blockIdx.x, q = blockIdx.y, Q = gridDim.y, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  int qa, qb;
  head_slice(N2 >> 2, Q, q, qa, qb);
  const int ncol = qb - qa;
  const int c = tid & (HS - 1), g = tid >> 5;
  constexpr int JU = 13;
  f32x4 w[JU];
  if (!(SKIP & 4)) {
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * j + g;
      w[j] = (o < C && c < ncol) ? *reinterpret_cast<const f32x4*>(W3 + (int64_t)o * ldw3 + 4 * (qa + c))
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  f32x4 hh = {0.f, 0.f, 0.f, 0.f};
  if (tid < ncol) hh = reinterpret_cast<const f32x4*>(h2 + (int64_t)m * N2)[qa + tid];
  for (int o = tid; o < C; o += 256) {
    float v = b3 ? b3[o] : 0.f;
    if (!(SKIP & 1)) {
#pragma unroll 8
      for (int s = 0; s < Qp; ++s) v += plog[((int64_t)s * M + m) * C + o];
    }
    lg[o] = v;
  }
  __syncthreads();
  const int64_t lab = y[m];
  if (!(SKIP & 2) && wv == 0) {
    float mx = -INFINITY;
    for (int cc = lane; cc < C; cc += 64) mx = fmaxf(mx, lg[cc]);
    mx = sl_wave_max(mx);
    float se = 0.f;
    for (int cc = lane; cc < C; cc += 64) se += expf(lg[cc] - mx);
    se = sl_wave_sum(se);
    if (lane == 0 && q == 0) loss_rows[m] = mx + logf(se) - lg[lab];
    const float inv = 1.f / se;
    for (int cc = lane; cc < C; cc += 64) {
      float p = expf(lg[cc] - mx) * inv;
      if (cc == lab) p -= 1.f;
      lg[cc] = p * scale;
    }
  }
  __syncthreads();
  if (q == 0)
    for (int cc = tid; cc < C; cc += 256) dlog[(int64_t)m * C + cc] = lg[cc];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (!(SKIP & 4)) {
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const int o = 8 * j + g;
      const float l = o < C ? lg[o] : 0.f;
      acc += l * w[j];
    }
  }
  part[g][c] = acc;
  __syncthreads();
  if (tid < ncol) {
    f32x4 v = part[0][tid];
#pragma unroll
    for (int gg = 1; gg < 8; ++gg) v += part[gg][tid];
    f32x4 out;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = hh[i] > 0.f ? v[i] * dscale : 0.f;
    reinterpret_cast<f32x4*>(dz2 + (int64_t)m * N2)[qa + tid] = out;
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// GPU time per launch: N launches captured in one hipGraph, replayed R times (no host
// launch cost in the measurement).  cold: each launch behind a 512 MB memset inside the
// graph, minus a graph of the memsets alone.
template <class F>
static float graph_us(F f, int n, int reps, void* flush, size_t fbytes, bool cold) {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  g_probe_stream = s;
  for (int i = 0; i < n; ++i) {
    if (cold) (void)hipMemsetAsync(flush, i & 0xff, fbytes, s);
    f();
  }
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, s);
  for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(s);
  return ms * 1000.f / (n * reps);
}

int main() {
  const int M = 16, N2 = 1000, C = 100, S2 = 16;
  int Q = head3_slices(N2);
  const int64_t slab2 = (int64_t)M * N2;
  float *P2, *W3, *b2, *b3, *h2, *ws, *dlog, *dz2, *loss, *scratch;
  int64_t* y;
  void* flush;
  const size_t fbytes = 512ull << 20;
  CK(hipMalloc(&P2, sizeof(float) * S2 * slab2));
  CK(hipMalloc(&W3, sizeof(float) * C * N2));
  CK(hipMalloc(&b2, sizeof(float) * N2));
  CK(hipMalloc(&b3, sizeof(float) * C));
  CK(hipMalloc(&h2, sizeof(float) * M * N2));
  CK(hipMalloc(&ws, sizeof(float) * 64 * M * C));
  CK(hipMalloc(&dlog, sizeof(float) * M * C));
  CK(hipMalloc(&dz2, sizeof(float) * M * N2));
  CK(hipMalloc(&loss, sizeof(float) * M));
  CK(hipMalloc(&scratch, sizeof(float) * 16));
  CK(hipMalloc(&y, sizeof(int64_t) * M));
  CK(hipMalloc(&flush, fbytes));
  std::vector<float> hp(S2 * slab2), hw(C * N2), hb(N2, 0.01f), hb3(C, 0.f);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.4f;
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (float)((i * 40503u) % 1000) / 30000.f - 0.015f;
  std::vector<int64_t> hy(M);
  for (int i = 0; i < M; ++i) hy[i] = i % 10;
  CK(hipMemcpy(P2, hp.data(), sizeof(float) * hp.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(W3, hw.data(), sizeof(float) * hw.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(b2, hb.data(), sizeof(float) * N2, hipMemcpyHostToDevice));
  CK(hipMemcpy(b3, hb3.data(), sizeof(float) * C, hipMemcpyHostToDevice));
  CK(hipMemcpy(y, hy.data(), sizeof(int64_t) * M, hipMemcpyHostToDevice));
  CK(hipMemset(scratch, 0, sizeof(float) * 16));
  // fc2 forward / dgrad at the TP = 1 server-step shape: W2 [1000, 5000], h1 / dz1 [16, 5000]
  const int K1 = 5000;
  float *W2, *h1, *dz1, *dgws, *fws, *dz2in;
  CK(hipMalloc(&W2, sizeof(float) * N2 * K1));
  CK(hipMalloc(&h1, sizeof(float) * M * K1));
  CK(hipMalloc(&dz1, sizeof(float) * M * K1));
  CK(hipMalloc(&dgws, sizeof(float) * 16 * M * K1));
  CK(hipMalloc(&fws, sizeof(float) * 16 * M * N2));
  CK(hipMalloc(&dz2in, sizeof(float) * M * N2));
  CK(hipMemset(W2, 0, sizeof(float) * N2 * K1));
  CK(hipMemset(h1, 0, sizeof(float) * M * K1));
  CK(hipMemset(dz2in, 0, sizeof(float) * M * N2));
  Epi e2{};
  e2.bias = b2;
  e2.relu = 1;
  e2.thresh = 0x80000000u;
  e2.dscale = 2.f;
  e2.seed_lo = 1;
  e2.seed_hi = 2;

  auto k_empty = [&] { empty_kernel<<<1, 64, 0, g_probe_stream>>>(scratch); };
  auto k_empty256 = [&] { empty_kernel<<<256, 256, 0, g_probe_stream>>>(scratch); };
  auto k_fwd = [&] {
    head_fwd_kernel<false><<<dim3(M, Q), 256, 0, g_probe_stream>>>(P2, S2, slab2, e2, W3, N2, h2, ws, M, N2, C);
  };
  auto k_bwd = [&] {
    head_bwd_kernel<false><<<dim3(M, Q), 256, (size_t)C * sizeof(float), g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M,
                                                                               2.f, h2, dlog, dz2, loss, M, N2, C, Q);
  };
  auto k_fwd0 = [&] {
    head_fwd_v0_kernel<<<dim3(M, Q), 256, 0, g_probe_stream>>>(P2, S2, slab2, e2, W3, N2, h2, ws, M, N2, C, 0);
  };
  auto k_bwd0 = [&] {
    head_bwd_v0_kernel<<<dim3(M, Q), 256, (size_t)C * sizeof(float), g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M,
                                                                           2.f, h2, dlog, dz2, loss, M, N2, C, 0, Q);
  };
  auto k_pair0 = [&] {
    k_fwd0();
    k_bwd0();
  };
  auto k_pair = [&] {
    k_fwd();
    k_bwd();
  };
  const int Qm = head3m_slices(N2);
  auto k_fwd_m = [&] {
    head_fwd_mfma_kernel<<<Qm, 256, 0, g_probe_stream>>>(P2, S2, slab2, e2, W3, N2, h2, ws, M, N2, C, 0);
  };
  auto k_pair_m = [&] {
    k_fwd_m();
    head_bwd_kernel<false><<<dim3(M, 8), 256, (size_t)C * sizeof(float), g_probe_stream>>>(ws, b3, W3, N2, y, -100,
                                                                                          1.f / M, 2.f, h2, dlog, dz2,
                                                                                          loss, M, N2, C, Qm);
  };
  auto k_pair_mm = [&] {
    k_fwd_m();
    head_bwd_mfma_kernel<<<Qm, 256, 0, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M,
                                                         N2, C, 0, Qm);
  };
  auto k_bwd_mm = [&] {
    head_bwd_mfma_kernel<<<Qm, 256, 0, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M,
                                                         N2, C, 0, Qm);
  };
  auto k_dgrad = [&] {
    skinny_dgrad_kernel<8><<<dim3(79, 1, 8), 512, 0, g_probe_stream>>>(dz2in, N2, W2, K1, nullptr, 0, 1.f, dgws, 0,
                                                                       (int64_t)M * K1, M, N2, K1);
  };
  auto k_dred = [&] {
    dgrad_reduce_kernel<<<(M * K1 + 255) / 256, 256, 0, g_probe_stream>>>(dgws, 8, (int64_t)M * K1, h1, K1, 2.f, dz1,
                                                                          K1, M, K1);
  };
  auto k_dgrad_pair = [&] {
    k_dgrad();
    k_dred();
  };
  auto k_fwd2 = [&] {
    skinny_fwd_once_kernel<4><<<dim3(63, 1, 10), 512, 0, g_probe_stream>>>(h1, K1, W2, K1, fws, N2, M, N2, K1, e2, fws,
                                                                           (int64_t)M * N2);
  };
  auto k_fwd_dgrad = [&] {
    k_fwd2();
    k_dgrad_pair();
  };
  auto bwdp = [&](int skip) {
    return [&, skip] {
      const size_t sh = (size_t)C * sizeof(float);
      switch (skip) {
        case 1: head_bwd_part<1><<<dim3(M, Q), 256, sh, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M, N2, C, Q); break;
        case 2: head_bwd_part<2><<<dim3(M, Q), 256, sh, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M, N2, C, Q); break;
        case 4: head_bwd_part<4><<<dim3(M, Q), 256, sh, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M, N2, C, Q); break;
        case 7: head_bwd_part<7><<<dim3(M, Q), 256, sh, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M, N2, C, Q); break;
        default: head_bwd_part<0><<<dim3(M, Q), 256, sh, g_probe_stream>>>(ws, b3, W3, N2, y, -100, 1.f / M, 2.f, h2, dlog, dz2, loss, M, N2, C, Q); break;
      }
    };
  };
  auto k_p1 = [&] { head_fwd_part<1><<<dim3(M, Q), 256, 0, g_probe_stream>>>(P2, S2, slab2, e2, W3, N2, h2, ws, M, N2, C); };
  auto k_p2 = [&] { head_fwd_part<2><<<dim3(M, Q), 256, 0, g_probe_stream>>>(P2, S2, slab2, e2, W3, N2, h2, ws, M, N2, C); };
  struct Row {
    const char* name;
    std::function<void()> f;
  };
  std::vector<Row> rows = {{"empty 1 WG", k_empty},      {"empty 256 WG", k_empty256}, {"head_fwd", k_fwd},
                           {"head_bwd", k_bwd},          {"head pair", k_pair}, {"head_fwd v0", k_fwd0}, {"head_bwd v0", k_bwd0}, {"head pair v0", k_pair0},        {"head_fwd slab phase", k_p1},
                           {"head_fwd logits phase", k_p2}, {"head_fwd_mfma", k_fwd_m},
                           {"head pair (fwd_mfma)", k_pair_m},
                           {"head_bwd_mfma", k_bwd_mm}, {"head pair (both mfma)", k_pair_mm},
                           {"fc2 dgrad (split-N 8)", k_dgrad}, {"fc2 dgrad reduce", k_dred},
                           {"fc2 dgrad + reduce", k_dgrad_pair}, {"fc2 fwd (once, S 10)", k_fwd2},
                           {"fc2 fwd + dgrad + reduce", k_fwd_dgrad},
                           {"head_bwd copy", bwdp(0)}, {"head_bwd no plog reduce", bwdp(1)},
                           {"head_bwd no softmax", bwdp(2)}, {"head_bwd no dz2 phase", bwdp(4)},
                           {"head_bwd skeleton", bwdp(7)}};
  for (int qv : {8}) {
    Q = qv;
    printf("Q = %d column slices\n", Q);
    for (auto& r : rows) {
      if (Q != 8 && r.name[0] == 'e') continue;
      const float hot = graph_us(r.f, 50, 20, flush, fbytes, false);
      const float cold = graph_us(r.f, 20, 5, flush, fbytes, true) - graph_us([] {}, 20, 5, flush, fbytes, true);
      const size_t wb = 48ull << 20;
      const float warm = graph_us(r.f, 20, 5, flush, wb, true) - graph_us([] {}, 20, 5, flush, wb, true);
      printf("  %-26s hot %7.2f us   warm %7.2f us   cold %7.2f us   (GPU time per launch, graph replay)\n", r.name,
             hot, warm, cold);
    }
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
