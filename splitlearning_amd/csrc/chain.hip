// The server step's latency chain as ONE persistent launch.
//
// Reference: the forward and backward of bob.train_and_backward's step
// (data_entities_vanilla_sisa.py:298-313, model2_sisa = fc1 -> ReLU -> dropout -> fc2 -> ReLU ->
// dropout -> fc3, models.py) between two optimizer steps: everything of the step except the
// wgrad + Adam stream, which stays in wgrad_group_kernel (fused.hip) because it is
// bandwidth-bound and already at the streaming roofline (docs/PERF.md).
//
// The launch-per-stage executor runs this part as six kernels (fc1 epilogue, fc2 split-K
// forward, head_fwd, head_bwd, fc2 dgrad, dgrad reduce).  Each moves little data (W2 twice, 20 MB
// at TP = 1) but pays a kernel boundary (~1.5-1.9 us, MI355X_MICROARCH.md) and a ramp, so
// together they take ~36 us of a 173 us TP = 1 step.  Here one launch of G workgroups (one
// per CU) runs the same math with in-launch hand-offs.  Each hand-off is the seam of
// resident.hip: write-through (sc1) payload stores, every wave drains, one agent-scope
// counter add per workgroup, consumers poll and then read with sc1 loads.
//
// Roles (a workgroup can hold several):
//   tile (rb, cb), 8 x NCB of them: W2[r0 .. r0 + WR)[c0 .. c0 + WC), at most 128 x 160,
//        loaded once into LDS and used by both products.  The 8 row blocks of column block cb
//        are workgroups cb, cb + NCB, ..., i.e. one XCD's L2 when NCB % 8 == 0.
//        F1  h1 rows {rb, rb + 8} of the slice: the look-ahead slabs summed in a fixed order,
//            plus bias, ReLU and dropout (engine.cpp linear_epilogue's math).  Stored to h1;
//            the column group exchanges them (group counter 0).
//        F4  fc2 partial FP[cb][m][r0 + n] = h1[m, slice] . W2[r0 + n, slice]
//            (exact-fp32 MFMA 16x16x4; one wave per 16 rows)                    -> seam 0
//   head w < N2 / 4: fc2 rows 4w .. 4w + 3.
//        H   P2 = the NCB partials in order; tensor-parallel: the peer-mapped granule exchange
//            of resident.hip, summed in rank order; then h2 = drop(relu(P2 + b2)) and the
//            logit partials of these rows                                       -> seam 1
//   softmax w < M: row w's logits (partials in order, + b3), softmax-CE, dlogits and loss
//                                                                                -> seam 2
//   head (again): dh2 = dlogits . W3[:, rows], then dz2 via the ReLU / dropout mask
//                                                                                -> seam 3
//   tile (again): dz1 partial over its rows, DP[rb][m][slice] (MFMA).  Group counter 1, then
//        rows {rb, rb + 8} of the slice: the 8 partials in order, h1 > 0 mask, dropout scale
//        -> dz1.
// Summation orders are fixed, so a launch is deterministic.  They differ from the six-kernel
// path, so results agree with it to fp32 rounding, not bitwise (tests/test_chain_gpu.py).
// Every wait is bounded (wall clock).  A timeout raises err, and every later wait gives up
// at once.  The host checks co-residency (chain_max_workgroups) and reads err after the epoch.
#include "chain.h"

namespace sl {

namespace {

typedef int ch_i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ch_rs(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
// hand-off traffic: write-through (sc1) stores, L1-bypassing (sc1) loads (aux 16)
__device__ __forceinline__ f32x4 ch_ld4(__amdgpu_buffer_rsrc_t rs, int boff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 16));
}
__device__ __forceinline__ void ch_st4(__amdgpu_buffer_rsrc_t rs, int boff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ch_i32x4, v), rs, boff, 0, 16);
}
__device__ __forceinline__ void ch_st1(__amdgpu_buffer_rsrc_t rs, int boff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rs, boff, 0, 16);
}

__device__ __forceinline__ unsigned ch_poll(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool ch_failed(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// every wave drains its write-through stores, the barrier orders the drains before thread 0's add
__device__ __forceinline__ void ch_arrive(unsigned* c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded poll of one counter until it reaches tgt; false when it gave up
__device__ __forceinline__ bool ch_spin(const ChainArgs& a, const unsigned* p, unsigned tgt) {
  if (ch_poll(p) >= tgt) return true;
  const uint64_t t0 = wall_clock64();
  while (ch_poll(p) < tgt) {
    if (ch_failed(a.err)) return false;
    __builtin_amdgcn_s_sleep(1);
    if ((int64_t)(wall_clock64() - t0) > a.timeout) {
      __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ unsigned* ch_seam(const ChainArgs& a, int seam, int shard) {
  return a.cnt + (seam * 8 + shard) * kChStride;
}
__device__ __forceinline__ unsigned* ch_group(const ChainArgs& a, int set, int cb) {
  return a.cnt + (kChSeams * 8 + set * kChMaxCB + cb) * kChStride;
}

// every shard of `seam` holds this launch's arrivals (lanes 0..7 of wave 0 poll one shard
// each); uniform result over the workgroup
__device__ __forceinline__ bool ch_seam_wait(const ChainArgs& a, int seam, int* s_ok) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < 8) {
      const int n = a.shard_n[seam * 8 + lane];
      if (n > 0) ok = ch_spin(a, ch_seam(a, seam, lane), a.gen * (unsigned)n);
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return *s_ok != 0;
}

__device__ __forceinline__ bool ch_group_wait(const ChainArgs& a, int set, int cb, int* s_ok) {
  if (threadIdx.x == 0) *s_ok = ch_spin(a, ch_group(a, set, cb), a.gen * (unsigned)kChRB) ? 1 : 0;
  __syncthreads();
  return *s_ok != 0;
}

// LDS carve (bytes, multiples of 16)
constexpr int kPW = 4 * kChMaxWC4 + 1;                 // W2 tile / h1 slice row pitch (floats)
constexpr int kPD = kChMaxWR + 1;                      // dz2 slice row pitch
constexpr int OFF_W2 = 0;                              // W2 tile [kChMaxWR][kPW]
constexpr int OFF_H1 = OFF_W2 + ((kChMaxWR * kPW * 4 + 15) & ~15);    // h1 slice [16][kPW]
constexpr int OFF_DZ = OFF_H1 + ((16 * kPW * 4 + 15) & ~15);          // dz2 slice [16][kPD]
constexpr int OFF_RED = OFF_DZ + ((16 * kPD * 4 + 15) & ~15);         // [16][32] f32x4
constexpr int OFF_W3 = OFF_RED + 16 * 32 * 16;         // W3 columns of the head rows [4][kChMaxC]
constexpr int OFF_DL = OFF_W3 + 4 * kChMaxC * 4;       // dlogits [16][kChMaxC]
constexpr int OFF_H2 = OFF_DL + 16 * kChMaxC * 4;      // h2 [16][4]
constexpr int OFF_DZH = OFF_H2 + 16 * 4 * 4;           // dz2 of the head rows [16][4]
constexpr int OFF_P2 = OFF_DZH + 16 * 4 * 4;           // P2 of the head rows [16] f32x4
constexpr int OFF_OK = OFF_P2 + 16 * 16;
constexpr int kChLds = OFF_OK + 16;
static_assert(kChLds <= 160 * 1024, "LDS");

}  // namespace

// phase timestamp k (workgroups 0 and G - 1, thread 0; only when a.trace is set)
#define CH_MARK(k)                                                                            \
  do {                                                                                        \
    if (a.trace != nullptr && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1)) \
      a.trace[(blockIdx.x == 0 ? 0 : 16) + (k)] = (int64_t)wall_clock64();                   \
  } while (0)

__global__ void __launch_bounds__(kChThreads) chain_step_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sw2 = reinterpret_cast<float*>(smem + OFF_W2);
  float* sh1 = reinterpret_cast<float*>(smem + OFF_H1);
  float* sdz = reinterpret_cast<float*>(smem + OFF_DZ);
  f32x4* red = reinterpret_cast<f32x4*>(smem + OFF_RED);
  float* sW3 = reinterpret_cast<float*>(smem + OFF_W3);
  float* sdl = reinterpret_cast<float*>(smem + OFF_DL);
  float* sh2 = reinterpret_cast<float*>(smem + OFF_H2);
  float* sdzh = reinterpret_cast<float*>(smem + OFF_DZH);
  f32x4* sp2 = reinterpret_cast<f32x4*>(smem + OFF_P2);
  int* s_ok = reinterpret_cast<int*>(smem + OFF_OK);
  constexpr int MC = kChMaxC;
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  CH_MARK(0);

  const int w = blockIdx.x, tid = threadIdx.x;
  const int r = tid >> 6, lane = tid & 63, li = lane & 15, lq = lane >> 4;
  const int M = a.M, N1 = a.N1, N2 = a.N2, C = a.C, C4 = a.C4, NCB = a.NCB;
  const bool tile = w < kChRB * NCB, head = w < a.HW;
  const int rb = tile ? w / NCB : 0, cb = tile ? w - rb * NCB : 0;
  // tile ranges: rows in groups of 4, columns in float4
  const int Q2 = N2 >> 2, Q4 = N1 >> 2;
  const int g0 = rb * Q2 / kChRB, g1 = (rb + 1) * Q2 / kChRB;
  const int r0 = 4 * g0, WR = 4 * (g1 - g0);
  const int q0 = cb * Q4 / NCB, q1 = (cb + 1) * Q4 / NCB;
  const int c0 = 4 * q0, WC4 = q1 - q0, WC = 4 * WC4;
  const __amdgpu_buffer_rsrc_t rH1 = ch_rs(a.h1), rFP = ch_rs(a.FP), rLP = ch_rs(a.LP), rDL = ch_rs(a.DL),
                               rDZ2 = ch_rs(a.dz2), rDP = ch_rs(a.DP);

  // Loads in the order they are consumed (a wave's loads complete in order, so consuming one
  // waits for every load issued before it; W2's block issued first held the slab sums until
  // it had arrived, 10.6 us measured): the look-ahead slabs of this workgroup's two h1 rows
  // {rb, rb + 8} of the slice (6 slab groups x 2 rows x WC4 float4, <= 4 per thread), then the
  // tile's W2 block (first needed after h1 is formed and exchanged), then the head rows' W3
  // columns (one float per thread, into LDS at the head phase)
  constexpr int EW = 2 * kChMaxWC4, SG = kChThreads / EW, SPT = kChMaxSlabs / SG;   // 80 x 6, 4
  const int e1 = tid % EW, sg1 = tid / EW;
  const int k1 = e1 / max(WC4, 1), qe1 = e1 - k1 * max(WC4, 1), m1 = rb + kChRB * k1;
  const bool act1 = tile && tid < SG * EW && k1 < 2 && m1 < M && WC4 > 0;
  f32x4 sl[SPT];
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    const int sb = sg1 + SG * u;
    sl[u] = (act1 && sb < a.S1)
                ? *reinterpret_cast<const f32x4*>(a.pn + (int64_t)sb * a.slab + (int64_t)m1 * N1 + c0 + 4 * qe1)
                : zv;
  }
  constexpr int U2 = kChMaxWR * kChMaxWC4 / kChThreads;
  f32x4 wv[U2];
#pragma unroll
  for (int u = 0; u < U2; ++u) {
    const int e = tid + u * kChThreads;
    const int row = e / max(WC4, 1), q = e - row * max(WC4, 1);
    wv[u] = (tile && row < WR && WC4 > 0)
                ? *reinterpret_cast<const f32x4*>(a.W2 + (int64_t)(r0 + row) * N1 + c0 + 4 * q)
                : zv;
  }
  static_assert(4 * MC == kChThreads, "one W3 element per thread");
  float w3r = 0.f;
  {
    const int ii = tid / MC, c = tid - ii * MC;
    if (head && c < C) w3r = a.W3[(int64_t)c * N2 + 4 * w + ii];
  }

  // ================= F: h1 slice, fc2 partial products
  if (tile) {
    // F1: h1 rows {rb, rb + 8} of the slice: the slab groups' sums in group order, bias,
    // ReLU, dropout (engine.cpp linear_epilogue's math) -> h1, exchanged within the column
    // group (its 8 workgroups share one XCD's L2 when NCB % 8 == 0)
    {
      f32x4 v = sl[0];
#pragma unroll
      for (int u = 1; u < SPT; ++u) v += sl[u];
      if (tid < SG * EW) red[sg1 * EW + e1] = v;
    }
    __syncthreads();
    if (tid < 2 * WC4) {
      const int kk = tid / WC4, qq = tid - kk * WC4;
      const int mm = rb + kChRB * kk;
      if (mm < M) {
        f32x4 s = red[tid];
#pragma unroll
        for (int g = 1; g < SG; ++g) s += red[g * EW + tid];
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = apply_epi(a.e1, s[i], mm, c0 + 4 * qq + i);
        ch_st4(rH1, ((mm * N1) + c0 + 4 * qq) * 4, o);
      }
    }
    ch_arrive(ch_group(a, 0, cb));
    CH_MARK(1);
    if (!ch_group_wait(a, 0, cb, s_ok)) return;
    CH_MARK(2);
    // F2: the whole h1 slice (rows >= M zero) -> LDS
    for (int e = tid; e < 16 * WC4; e += kChThreads) {
      const int m = e / WC4, q = e - m * WC4;
      const f32x4 v = m < M ? ch_ld4(rH1, ((m * N1) + c0 + 4 * q) * 4) : zv;
#pragma unroll
      for (int i = 0; i < 4; ++i) sh1[m * kPW + 4 * q + i] = v[i];
    }
    // F3: the W2 block -> LDS
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int e = tid + u * kChThreads;
      const int row = e / max(WC4, 1), q = e - row * max(WC4, 1);
      if (row < kChMaxWR)
#pragma unroll
        for (int i = 0; i < 4; ++i) sw2[row * kPW + 4 * q + i] = wv[u][i];
    }
    __syncthreads();
    CH_MARK(3);
    // F4: wave r: rows 16 r .. 16 r + 15 of the tile, K = the slice
    if (16 * r < WR) {
      // two accumulators (even / odd k steps) so consecutive MFMAs do not wait on each other
      f32x4 acc0 = zv, acc1 = zv;
      const float* pa = sh1 + li * kPW + lq;
      const float* pb = sw2 + (16 * r + li) * kPW + lq;
#pragma unroll
      for (int kk = 0; kk < kChMaxWC4; kk += 2) {
        if (kk < WC4) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * kk], pb[4 * kk], acc0, 0, 0, 0);
        if (kk + 1 < WC4) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * kk + 4], pb[4 * kk + 4], acc1, 0, 0, 0);
      }
      const f32x4 acc = acc0 + acc1;
      const int n = 16 * r + li;
      if (n < WR)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 4 * lq + i;
          if (m < M) ch_st1(rFP, (((cb * 16 + m) * N2) + r0 + n) * 4, acc[i]);
        }
    }
    ch_arrive(ch_seam(a, 0, w & 7));
    CH_MARK(4);
  }

  // ================= H: P2 of the head rows, h2, logit partials
  if (head) {
    sW3[tid] = w3r;                              // ordered before its readers by the wait's barrier
    if (!ch_seam_wait(a, 0, s_ok)) return;
    CH_MARK(5);
    {
      const int m = tid >> 5, cq = tid & 31;
      red[m * 32 + cq] = (m < M && cq < NCB) ? ch_ld4(rFP, (((cq * 16 + m) * N2) + 4 * w) * 4) : zv;
    }
    __syncthreads();
    if (tid < 16) {
      f32x4 s = red[tid * 32];
#pragma unroll
      for (int cq = 1; cq < kChMaxCB; ++cq) s += red[tid * 32 + cq];   // partials >= NCB are zero
      sp2[tid] = s;
    }
    __syncthreads();
    if (tid < 64) {
      const int m = tid >> 2, ii = tid & 3;
      float pv = sp2[m][ii];
      if (a.ipc.T > 0) {
        // tensor-parallel fc2 (row-parallel): the 16 x 4 block to every rank as 8-byte
        // granules {generation, value} (the data is its own flag), summed in rank order on
        // every rank (resident.hip's exchange; region reuse is ordered by the exchange itself)
        const uint32_t gen = a.ipc.gen;
        const int ipar = (int)(gen & 1u), T = a.ipc.T, me = a.ipc.me;
        const int64_t half = a.ipc.cap >> 1;
        const int64_t slot = (int64_t)w * 64 + tid;
        const uint64_t gr = ((uint64_t)gen << 32) | (uint64_t)__builtin_bit_cast(uint32_t, pv);
        for (int rr = 0; rr < T; ++rr)
          __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ipc.P.data[rr]) + (ipar * T + me) * half + slot, gr,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t* mine = reinterpret_cast<const uint64_t*>(a.ipc.P.data[me]);
        bool ok = true;
        float sum = 0.f;
        for (int src = 0; src < T && ok; ++src) {
          const uint64_t* g = mine + (ipar * T + src) * half + slot;
          uint64_t x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((uint32_t)(x >> 32) != gen) {
            const uint64_t t0 = wall_clock64();
            while ((uint32_t)((x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >> 32) != gen) {
              if (__hip_atomic_load(a.ipc.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                ok = false;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
              if ((int64_t)(wall_clock64() - t0) > a.ipc.timeout) {
                ipc_fail(a.ipc.err, a.ipc.herr);
                ok = false;
                break;
              }
            }
          }
          sum += __builtin_bit_cast(float, (uint32_t)(x & 0xffffffffull));
        }
        ok = __all(ok);
        if (!ok && tid == 0) __hip_atomic_fetch_or(a.err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pv = sum;
        if (tid == 0) *s_ok = ok ? 1 : 0;
      }
      const int n = 4 * w + ii;
      float h = 0.f;
      if (m < M) {
        h = apply_epi(a.e2, pv, m, n);
        a.h2[(int64_t)m * N2 + n] = h;
      }
      sh2[m * 4 + ii] = h;
    }
    __syncthreads();
    if (a.ipc.T > 0 && *s_ok == 0) return;
    {
      const int nc4 = C4 >> 2;
      if (tid < 16 * nc4) {
        const int m = tid / nc4, c = 4 * (tid - m * nc4);
        if (m < M) {
          f32x4 v = zv;
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) v += sh2[m * 4 + ii] * *reinterpret_cast<const f32x4*>(sW3 + ii * MC + c);
          ch_st4(rLP, (((w * 16 + m) * C4) + c) * 4, v);
        }
      }
    }
    ch_arrive(ch_seam(a, 1, w & 7));
    CH_MARK(6);
  }

  // ================= S: row m's logits, softmax-CE, dlogits (workgroups m < M)
  if (w < M) {
    if (!ch_seam_wait(a, 1, s_ok)) return;
    CH_MARK(7);
    const int m = w;
    const int nc4 = C4 >> 2;
    constexpr int NG = kChThreads / 32;                   // 16 partial-sum groups
    {
      const int c4 = tid & 31, gq = tid >> 5;
      f32x4 v = zv;
      if (c4 < nc4) {
        f32x4 parts[256 / NG];
#pragma unroll
        for (int k = 0; k < 256 / NG; ++k) {
          const int src = gq + NG * k;
          parts[k] = src < a.HW ? ch_ld4(rLP, (((src * 16 + m) * C4) + 4 * c4) * 4) : zv;
        }
#pragma unroll
        for (int k = 0; k < 256 / NG; ++k) v += parts[k];
      }
      red[gq * 32 + c4] = v;
    }
    __syncthreads();
    if (tid < 64) {
      const int c4 = tid & 31;
      const bool act = tid < 32 && c4 < nc4;
      f32x4 lg = zv;
      if (act) {
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) lg += red[gq * 32 + c4];
#pragma unroll
        for (int i = 0; i < 4; ++i) lg[i] += (4 * c4 + i < C && a.b3) ? a.b3[4 * c4 + i] : 0.f;
      }
      const int64_t lab = a.Y[m];
      const bool ign = lab == a.ignore || lab < 0 || lab >= C;
      float mx = -INFINITY;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (act && 4 * c4 + c < C) mx = fmaxf(mx, lg[c]);
      mx = sl_wave_max(mx);
      f32x4 e = zv;
      float se = 0.f, zl = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = 4 * c4 + c;
        if (act && cc < C) {
          e[c] = expf(lg[c] - mx);
          se += e[c];
          if (cc == lab) zl = lg[c];
        }
      }
      se = sl_wave_sum(se);
      zl = sl_wave_sum(zl);
      const float inv = 1.f / se;
      f32x4 d = zv;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = 4 * c4 + c;
        float pr = e[c] * inv;
        if (cc == lab) pr -= 1.f;
        d[c] = (ign || cc >= C) ? 0.f : pr * a.ce_scale;
      }
      if (act) {
        ch_st4(rDL, ((m * C4) + 4 * c4) * 4, d);
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (4 * c4 + c < C) a.dlog[(int64_t)m * C + 4 * c4 + c] = d[c];
      }
      if (tid == 0) a.loss[m] = ign ? 0.f : mx + logf(se) - zl;
    }
    ch_arrive(ch_seam(a, 2, w & 7));
    CH_MARK(8);
  }

  // ================= B: dz2 of the head rows
  if (head) {
    if (!ch_seam_wait(a, 2, s_ok)) return;
    CH_MARK(9);
    // dlogits [16][MC] (rows >= M and classes >= C4 zero)
    for (int e = tid; e < 16 * (MC / 4); e += kChThreads) {
      const int m = e / (MC / 4), c = 4 * (e - m * (MC / 4));
      *reinterpret_cast<f32x4*>(sdl + m * MC + c) = (m < M && c < C4) ? ch_ld4(rDL, ((m * C4) + c) * 4) : zv;
    }
    __syncthreads();
    {
      // dh2[m][ii] = sum_c dlog[m][c] W3[c][4 w + ii]: 16 lanes per (m, ii)
#pragma unroll
      for (int oi0 = 0; oi0 < 64; oi0 += kChThreads / 16) {
        const int oi = oi0 + (tid >> 4), part = tid & 15;
        const int m = oi >> 2, ii = oi & 3;
        float s = 0.f;
#pragma unroll
        for (int c0 = 0; c0 < MC; c0 += 16) {
          const int c = c0 + part;
          s = fmaf(sdl[m * MC + c], sW3[ii * MC + c], s);
        }
        s = sl_row16_sum(s);
        if (part == 0) {
          const float h = sh2[m * 4 + ii];
          sdzh[m * 4 + ii] = (m < M && h > 0.f) ? s * a.e2.dscale : 0.f;
        }
      }
    }
    __syncthreads();
    if (tid < M) ch_st4(rDZ2, ((tid * N2) + 4 * w) * 4, *reinterpret_cast<const f32x4*>(sdzh + tid * 4));
    ch_arrive(ch_seam(a, 3, w & 7));
    CH_MARK(10);
  }

  // ================= D: dz1 of the tile's slice
  if (tile) {
    if (!ch_seam_wait(a, 3, s_ok)) return;
    CH_MARK(11);
    {
      const int m = tid >> 5, k4 = tid & 31;   // 16 rows x 32 float4 (kChMaxWR = 128)
      const f32x4 v = (m < M && 4 * k4 < WR) ? ch_ld4(rDZ2, ((m * N2) + r0 + 4 * k4) * 4) : zv;
#pragma unroll
      for (int i = 0; i < 4; ++i) sdz[m * kPD + 4 * k4 + i] = v[i];
    }
    __syncthreads();
    // wave r: column tiles jt = r and r + 8 of the slice (both in one K loop: the A operand is
    // shared and four accumulators keep consecutive MFMAs independent); K = the tile's rows
    {
      const int jt0 = r, jt1 = r + 8;
      const bool two = 16 * jt1 < WC;
      if (16 * jt0 < WC) {
        f32x4 a0 = zv, a1 = zv, b0 = zv, b1 = zv;
        const float* pa = sdz + li * kPD + lq;
        const float* pb0 = sw2 + lq * kPW + 16 * jt0 + li;
        const float* pb1 = sw2 + lq * kPW + 16 * (two ? jt1 : jt0) + li;
#pragma unroll
        for (int kk = 0; kk < kChMaxWR / 4; kk += 2) {
          if (4 * kk < WR) {
            const float x = pa[4 * kk];
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb0[4 * kk * kPW], a0, 0, 0, 0);
            if (two) b0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb1[4 * kk * kPW], b0, 0, 0, 0);
          }
          if (4 * kk + 4 < WR) {
            const float x = pa[4 * kk + 4];
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb0[(4 * kk + 4) * kPW], a1, 0, 0, 0);
            if (two) b1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb1[(4 * kk + 4) * kPW], b1, 0, 0, 0);
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (h == 1 && !two) break;
          const f32x4 acc = h == 0 ? a0 + a1 : b0 + b1;
          const int j = 16 * (h == 0 ? jt0 : jt1) + li;
          if (j < WC)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int m = 4 * lq + i;
              if (m < M) ch_st1(rDP, (((rb * 16 + m) * N1) + c0 + j) * 4, acc[i]);
            }
        }
      }
    }
    ch_arrive(ch_group(a, 1, cb));
    CH_MARK(12);
    if (!ch_group_wait(a, 1, cb, s_ok)) return;
    CH_MARK(13);
    if (tid < 2 * WC4) {
      const int k = tid / WC4, q = tid - k * WC4;
      const int m = rb + kChRB * k;
      if (m < M) {
        f32x4 parts[kChRB];
#pragma unroll
        for (int b = 0; b < kChRB; ++b) parts[b] = ch_ld4(rDP, (((b * 16 + m) * N1) + c0 + 4 * q) * 4);
        f32x4 v = parts[0];
#pragma unroll
        for (int b = 1; b < kChRB; ++b) v += parts[b];
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = sh1[m * kPW + 4 * q + i] > 0.f ? v[i] * a.s1 : 0.f;
        *reinterpret_cast<f32x4*>(a.dz1 + (int64_t)m * N1 + c0 + 4 * q) = o;
      }
    }
  }
  CH_MARK(14);
}
#undef CH_MARK

std::string chain_check(const ChainArgs& a) {
  if (a.M < 1 || a.M > 16) return "rows per step 1..16";
  if (a.N2 < 4 || a.N2 % 4 || a.N2 > 4 * kChRB * (kChMaxWR / 4) || a.HW != a.N2 / 4 || a.HW > a.G)
    return "fc2 width % 4, <= 1024 and <= 4 x workgroups";
  if (a.N1 < 4 || a.N1 % 4) return "fc1 shard width % 4";
  if (a.NCB < 1 || a.NCB > kChMaxCB || kChRB * a.NCB > a.G) return "column blocks";
  if ((a.N1 / 4 + a.NCB - 1) / a.NCB > kChMaxWC4) return "fc1 shard too wide for the tiles";
  if (a.C < 1 || a.C > kChMaxC || a.C4 % 4 || a.C4 < a.C) return "classes <= 128";
  if (a.G < a.M || a.G > 1024) return "workgroups";
  if (a.S1 < 1 || a.S1 > kChMaxSlabs || a.slab < (int64_t)a.M * a.N1) return "look-ahead slabs";
  if (a.ipc.T > 0 && ((int64_t)a.HW * 64 * 2 > a.ipc.cap || a.ipc.T > kIpcMaxRanks))
    return "peer-mapped exchange region";
  return "";
}

int chain_max_workgroups(int device) {
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, device) != hipSuccess) return 0;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&chain_step_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kChLds) != hipSuccess)
    return 0;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(&chain_step_kernel),
                                                   kChThreads, kChLds) != hipSuccess)
    return 0;
  return nb * pr.multiProcessorCount;
}

hipError_t chain_step_launch(const ChainArgs& a, hipStream_t st) {
  if (!chain_check(a).empty()) return hipErrorInvalidValue;
  chain_step_kernel<<<a.G, kChThreads, kChLds, st>>>(a);
  return hipGetLastError();
}

}  // namespace sl
