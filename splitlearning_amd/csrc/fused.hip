// Server-step fusions for Bob's 3-layer tail (fc1 ReLU+Dropout, fc2 ReLU+Dropout, fc3 ->
// cross-entropy; reference model2_sisa, models.py:46-63, trained per batch with Adam or SGD-m).
//
// At B = 16 the step is HBM-bound in fc1/fc2 and launch-bound everywhere else: the eager
// chain is 13 kernels, each with a ~1.5-2.5 us dependent-launch boundary, and on a
// tensor-parallel shard (1/8 of the bytes) the boundaries dominate.  Two fusions:
//
//  server_head3  two kernels over (row, 128-column slice) workgroups: reduce fc2's split-K
//                partial slabs + fc2's bias/ReLU/dropout (-> h2) + partial fc3 logits; then
//                logits, softmax-CE (loss, dlogits), fc3 data gradient and fc2's
//                ReLU/dropout backward (-> dz2).  Replaces fc2-epilogue, fc3-forward,
//                CE and fc3-dgrad.  (A one-workgroup-per-row version that recomputed the
//                logits per slice measured 59 us under rocprofv3: each workgroup streamed
//                all of W3 with dependent loads.  A one-workgroup-per-row version holding
//                its W3 share in registers, used for both the logits and dz2, measured
//                16.6 us against 14.4 us for these two kernels (TP = 1): one CU cannot pull
//                400 KB fast enough, W3 has to be spread over many CUs.)
//
//  wgrad_group_kernel   the fused wgrad+optimizer (v3 layout) for up to 3 layers in one
//                launch, plus (FWDN) fc1's look-ahead forward for the next batch.  (dZ given
//                as un-reduced split-N slabs, reduced while staging, measured slower than a
//                separate reduce launch at fc1's size: removed, docs/PERF.md.)
//
// The look-ahead SISA step is 7 launches: slab epilogue (h1), fc2 forward (split-K),
// head_fwd, head_bwd, fc2 dgrad (split-N) + reduce, wgrad_group.
#include "fused.h"

#include <algorithm>

namespace sl {

// Column slices of <= 32 float4 (128 columns) per workgroup; grid (M, Q) for both kernels.
constexpr int HS = 32;

// Head workgroup layout: grid (Q, M), slice q = float4 columns [32 q, 32 q + 32), so with
// Q = 8 dispatch slot L = q + 8 m runs on XCD q and slice q is exactly the 128 fc2 outputs
// whose W2 rows the XCD-grouped fc2 forward / dgrad keep on XCD q (csrc/linear.hip): the
// forward's slabs, h2 and dz2 of a slice stay in one XCD's L2 from the forward through
// head_fwd and head_bwd to the dgrad (L2 hit rate of the head kernels 66 -> 88 % against the
// earlier grid (M, Q) with proportional slices, profiles/r2_pmc_xcd_l2_hits.txt).
__device__ __forceinline__ void head_wg(int& m, int& q, int& Q) {
  q = blockIdx.x;
  m = blockIdx.y;
  Q = gridDim.x;
}

__device__ __forceinline__ void head_slice(int n4, int q, int& a, int& b) {
  a = min(n4, HS * q);
  b = min(n4, HS * q + HS);
}

// head_fwd_kernel: workgroup (m, q) reduces fc2's split-K slabs for its column slice of row
// m, applies fc2's epilogue (-> h2) and writes the slice's partial fc3 logits plog[q][m][:].
// Every load of a phase is issued before the first is consumed (one memory round trip per
// phase): at B = 16 this op is pure latency.  The per-output dot products over the slice's
// 32 float4 columns are reduced on DPP lane moves within each 16-lane row plus two
// v_readlane pairs (a 5-step ds_bpermute shuffle per output cost 2.6 us of the kernel in the
// graph-replay probe, scripts/probe/head_probe.hip).  BF: bf16 compute (operands rounded).
//
// IPC (tensor-parallel fc2, peer-mapped all-reduce fused in; ipc_ar.h): P2 is this rank's
// unreduced partial (S2 split-K slabs, summed first).  Wave 0 pushes the workgroup's slice of row m into slot [me] of every
// rank's region, drains its stores, raises flag (m, q) on every rank and waits for the T
// flags (m, q) of this generation; the slab reduction then reads the T slots (S2 = T, in rank
// order: bitwise the same sum on every rank).  One launch per step less than a separate
// all-reduce kernel, and the wait overlaps the W3 loads already in flight.
template <bool BF, bool IPC>
__global__ void __launch_bounds__(256)
head_fwd_kernel(const float* __restrict__ P2, int S2, int64_t slab2, Epi e2, const float* __restrict__ W3,
                int ldw3, float* __restrict__ h2, float* __restrict__ plog, int M, int N2, int C, IpcStep ip) {
  __shared__ f32x4 part[8][HS];
  __shared__ f32x4 hs[HS];
  int m, q, Q;
  head_wg(m, q, Q);
  const int tid = threadIdx.x;
  int qa, qb;
  head_slice(N2 >> 2, q, qa, qb);
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
  // the slab loads (consumed first) go out ahead of W3's (consumed after the reduction): a
  // wave's loads complete in order (non-IPC, S2 <= 16: two slabs per slab group).  Native
  // executor, us per server step: TP = 1 172.1 -> 170.3, TP = 8 52.6 -> 51.2 with head_bwd's
  // partial logits ahead of its W3 (profiles/r3h_head_load_order_ab.txt)
  const bool sfirst = !IPC && S2 <= 16;
  // gridDim.z > 1 (wide heads: SISA-concat's k x 100 logits, no IPC): workgroup z takes output
  // groups z, z + Z, ... (each group JU x 8 outputs); every z reduces the slabs, z = 0 stores h2
  const int j00 = JU * (int)blockIdx.z, jstep = JU * (int)gridDim.z;
  f32x4 sv0 = {0.f, 0.f, 0.f, 0.f}, sv1 = sv0;
  if (sfirst) {
    const int cc = tid & (HS - 1), sg = tid >> 5;
    if (cc < ncol) {
      const f32x4* src = reinterpret_cast<const f32x4*>(P2 + (int64_t)m * N2) + qa + cc;
      if (sg < S2) sv0 = src[sg * (slab2 >> 2)];
      if (sg + 8 < S2) sv1 = src[(sg + 8) * (slab2 >> 2)];
    }
  }
  load_w(j00);
  if constexpr (IPC) {
    __shared__ int s_ok;
    if (wv == 0) {
      if (lane < ncol) {
        // this rank's split-K slabs (S2 >= 1) summed in slab order: the plain product the
        // separate-launch path would all-reduce
        const f32x4* src = reinterpret_cast<const f32x4*>(P2 + (int64_t)m * N2) + qa + lane;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < S2; ++s) v += src[s * (slab2 >> 2)];
        const int64_t slot = ((int64_t)ip.par * ip.T + ip.me) * ip.cap + (int64_t)m * N2 + 4 * (qa + lane);
        for (int r = 0; r < ip.T; ++r) ipc_st4(ipc_rsrc(ip.P.data[r]), slot, make_float4(v[0], v[1], v[2], v[3]));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int fi = m * Q + q;
      if (lane < ip.T) ipc_raise_flag(ip.P.flags[lane] + ((int64_t)ip.par * ip.T + ip.me) * ip.nflags + fi, ip.gen, ip.fences);
      const bool ok = ipc_wait_flags(ip, lane, fi);
      if (lane == 0) s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    // a wait gave up (stalled / dead peer, error word raised): nothing sound to compute; the
    // job aborts on the error word (ServerEpoch::run polls its host mirror)
    if (!s_ok) return;
    P2 = ip.P.data[ip.me] + (int64_t)ip.par * ip.T * ip.cap;
    S2 = ip.T;
    slab2 = ip.cap;
  }
  // 1. slab reduction: 32 columns x 8 slab groups
  {
    const int cc = tid & (HS - 1), sg = tid >> 5;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (cc < ncol) {
      const f32x4* src = reinterpret_cast<const f32x4*>(P2 + (int64_t)m * N2) + qa + cc;
      if constexpr (IPC) {
        // the T slots of the peer-mapped region (S2 = T <= 8: one per slab group)
        const __amdgpu_buffer_rsrc_t rs = ipc_rsrc(ip.P.data[ip.me]);
        const int64_t o0 = (int64_t)ip.par * ip.T * ip.cap + (int64_t)m * N2 + 4 * (qa + cc);
        for (int s = sg; s < S2; s += 8) {
          const float4 u = ipc_ld4(rs, o0 + (int64_t)s * slab2);
          v += f32x4{u.x, u.y, u.z, u.w};
        }
      } else if (sfirst) {
        v += sv0;
        v += sv1;   // (zero when sg + 8 >= S2: the same sum as the loop below)
      } else {
#pragma unroll 4
        for (int s = sg; s < S2; s += 8) v += src[s * (slab2 >> 2)];
      }
    }
    part[sg][cc] = v;
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
      if (blockIdx.z == 0) reinterpret_cast<f32x4*>(h2 + (int64_t)m * N2)[qa + tid] = o;
    }
    hs[tid] = o;
  }
  __syncthreads();
  // 2. partial logits: half-wave h (32 lanes = the slice's columns) owns output 8 j + 2 wv + h
  const f32x4 h = BF ? bfr4(hs[c]) : hs[c];
  float* dst = plog + ((int64_t)q * M + m) * C;
  for (int j0 = j00; j0 * 8 < C; j0 += jstep) {
    if (j0 != j00) load_w(j0);
#pragma unroll
    for (int j = 0; j < JU; ++j) {
      const f32x4 wj = BF ? bfr4(w[j]) : w[j];
      const float d = sl_row16_sum(wj[0] * h[0] + wj[1] * h[1] + wj[2] * h[2] + wj[3] * h[3]);
      const float s0 = sl_lane(d, 0) + sl_lane(d, 16), s1 = sl_lane(d, 32) + sl_lane(d, 48);
      const int o = 8 * (j0 + j) + 2 * wv;
      if (lane == 0) {
        if (o < C) dst[o] = s0;
        if (o + 1 < C) dst[o + 1] = s1;
      }
    }
  }
}

// head_bwd_kernel: workgroup (m, q) sums row m's partial logits (+ b3), softmax-CE (loss and
// dlogits written by q == 0), then dz2 = (dlogits . W3) * dscale * [h2 > 0] for its slice.
// The softmax's two wave reductions run on DPP row moves + v_readlane, and each exponential
// is computed once (kept in LDS for the normalisation).  BF: bf16 compute.
template <bool BF>
__global__ void __launch_bounds__(256)
head_bwd_kernel(const float* __restrict__ plog, const float* __restrict__ b3, const float* __restrict__ W3,
                int ldw3, const int64_t* __restrict__ y, int64_t ignore, float scale, float dscale,
                const float* __restrict__ h2, float* __restrict__ dlog, float* __restrict__ dz2,
                float* __restrict__ loss_rows, int M, int N2, int C, int Qp, int G, const float* __restrict__ gscale) {
  // Qp: number of partial-logit slabs in plog (head_fwd: one per column slice)
  // G > 1: grouped cross-entropy (SISA-concat's k heads, protocols/concat.py): the C logits are
  // G groups of C / G, each with its own label y[m G + g], scale (gscale[m G + g] or `scale`) and
  // loss loss_rows[m G + g]; wave g % 4 takes group g
  extern __shared__ float lg[];   // C
  __shared__ f32x4 part[8][HS];
  int m, q, Q;
  head_wg(m, q, Q);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  int qa, qb;
  head_slice(N2 >> 2, q, qa, qb);
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
  // the partial logits (consumed first) load ahead of W3 and the h2 mask (C <= 256, Qp <= 8:
  // one output per thread; a wave's loads complete in order)
  const bool lfirst = C <= 256 && Qp <= 8;
  float pv[8];
  float b3v = 0.f;
  if (lfirst && tid < C) {
    b3v = b3 ? b3[tid] : 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) pv[s] = s < Qp ? plog[((int64_t)s * M + m) * C + tid] : 0.f;
  }
  load_w(0);
  f32x4 hh = {0.f, 0.f, 0.f, 0.f};
  if (tid < ncol) hh = reinterpret_cast<const f32x4*>(h2 + (int64_t)m * N2)[qa + tid];
  if (lfirst) {
    if (tid < C) {
      float v = b3v;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        if (s < Qp) v += pv[s];
      lg[tid] = v;
    }
  } else if (C <= 1024 && Qp <= 8) {
    // wide heads (SISA-concat's k x 100 logits): up to 4 outputs per thread, all 32 partial
    // loads in flight before the first sum (a loop per output took one round trip each), the
    // same sums in the same order
    float pw[4][8], bw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = tid + 256 * u;
      bw[u] = (o < C && b3) ? b3[o] : 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) pw[u][s] = (o < C && s < Qp) ? plog[((int64_t)s * M + m) * C + o] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = tid + 256 * u;
      float v = bw[u];
#pragma unroll
      for (int s = 0; s < 8; ++s)
        if (s < Qp) v += pw[u][s];
      if (o < C) lg[o] = v;
    }
  } else {
    for (int o = tid; o < C; o += 256) {
      float v = b3 ? b3[o] : 0.f;
#pragma unroll 8
      for (int s = 0; s < Qp; ++s) v += plog[((int64_t)s * M + m) * C + o];
      lg[o] = v;
    }
  }
  __syncthreads();
  const int Cg = C / G;
  for (int gr = wv; gr < G; gr += 4) {
    const int64_t lab = y[(int64_t)m * G + gr];
    float* lgg = lg + gr * Cg;
    const float sc = gscale ? gscale[(int64_t)m * G + gr] : scale;
    if (lab == ignore || lab < 0 || lab >= Cg) {
      for (int cc = lane; cc < Cg; cc += 64) lgg[cc] = 0.f;
      if (lane == 0 && q == 0) loss_rows[(int64_t)m * G + gr] = 0.f;
    } else {
      const float zl = lgg[lab];
      float mx = -INFINITY;
      for (int cc = lane; cc < Cg; cc += 64) mx = fmaxf(mx, lgg[cc]);
      mx = sl_wave_max_dpp(mx);
      float se = 0.f;
      for (int cc = lane; cc < Cg; cc += 64) {
        const float e = expf(lgg[cc] - mx);
        lgg[cc] = e;
        se += e;
      }
      se = sl_wave_sum_dpp(se);
      if (lane == 0 && q == 0) loss_rows[(int64_t)m * G + gr] = mx + logf(se) - zl;
      const float inv = 1.f / se;
      for (int cc = lane; cc < Cg; cc += 64) {
        float p = lgg[cc] * inv;
        if (cc == lab) p -= 1.f;
        lgg[cc] = p * sc;
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
      acc += BF ? bfr(l) * bfr4(w[j]) : l * w[j];
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

// Traversal order.  Workgroups are dispatched in linear (x fastest) order, so the tile
// order is the order in which fc1's W/m/v stream through the 256 MiB Infinity Cache.
// With grp.rev0 set, layer 0's tiles are walked last-to-first (the other layers keep
// their place at the end).  Alternating the direction every step makes the tiles one step
// touched last the ones the next step touches first: their lines are still resident
// (LRU reuse distance = the state streamed after them, not all 385 MB of it), so that
// part of the read+write stream is served on-die instead of by HBM.
// Tile mapping.  Either a 2-D grid (K blocks of the widest layer) x (row tiles of every
// layer), or a 1-D grid over the layers' real tiles, layer i owning blocks [wb0_i, wb0_i +
// ceil(N_i/16) * ceil(K_i/256)) in row-major tile order: the 2-D form leaves 55 % of its
// workgroups empty at a TP = 8 shard, where fc2's and fc3's K is 628 / 1000 against fc1's
// 5408 (the launcher picks the form, set_traversal's caller).  Layer 0's local index is
// reversed when grp.rev0 is set.  Every quantity is wave-uniform (readfirstlane on the
// quotient: the division itself is emitted on the VALU), so the layer descriptor stays in
// scalar registers.
__device__ __forceinline__ int wg_tile(const WgGroup& g, int& bx, int& by) {
  if (g.grid2d) {   // 2-D grid: (K blocks of the widest layer) x (row tiles of all layers)
    const int y = (int)blockIdx.y;
    const int layer = (g.n > 2 && y >= g.d[2].yb0) ? 2 : ((g.n > 1 && y >= g.d[1].yb0) ? 1 : 0);
    bx = (int)blockIdx.x;
    by = y - (layer == 2 ? g.d[2].yb0 : (layer == 1 ? g.d[1].yb0 : 0));
    if (layer == 0 && g.rev0) {
      bx = (int)gridDim.x - 1 - bx;
      by = (g.n > 1 ? g.d[1].yb0 : (int)gridDim.y) - 1 - by;
    }
    return layer;
  }
  const int lin = (int)blockIdx.x;
  const int li = (g.n > 2 && lin >= g.d[2].wb0) ? 2 : ((g.n > 1 && lin >= g.d[1].wb0) ? 1 : 0);
  const int wb0 = li == 2 ? g.d[2].wb0 : (li == 1 ? g.d[1].wb0 : 0);
  const int K = li == 2 ? g.d[2].K : (li == 1 ? g.d[1].K : g.d[0].K);
  const int kx = (K + 255) >> 8;
  int local = lin - wb0;
  if (li == 0 && g.rev0) local = g.nt0 - 1 - local;
  by = __builtin_amdgcn_readfirstlane(local / kx);
  bx = local - by * kx;
  return li;
}

// Write-through (sc1) 16-B store: the line leaves the XCD's L2 with the store, so the
// kernel does not end with up to 32 MB of dirty L2 lines for the next launch boundary to
// write back (default; variant 4 = 1: plain stores).  `boff` is the byte offset from `base` ([N, ld] floats).
__device__ __forceinline__ void st_wt(float* base, int N, int ld, int boff, f32x4 v) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, N * ld * 4, 0x00020000);
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rs, boff, 0, 16);
}

// Per-array cache-policy presets of the W / m / v stream (grp.pol, variant 21; buffer aux bits
// 0 plain, 2 non-temporal, 16 write-through): {W load, state load, W store, state store}.
// Preset 0 is the shipped form (plain loads, write-through stores).
__device__ __forceinline__ f32x4 ld_pol(const float* base, int bytes, int boff, int aux) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes, 0x00020000);
  if (aux == 2) return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 2));
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 0));
}
__device__ __forceinline__ void st_pol(float* base, int bytes, int boff, f32x4 v, int aux) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
  if (aux == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rs, boff, 0, 2);
  else if (aux == 16) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rs, boff, 0, 16);
  else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rs, boff, 0, 0);
}
__device__ __forceinline__ void pol_aux(int pol, int& lw, int& ls, int& sw, int& ss) {
  switch (pol) {
    case 1: lw = 0; ls = 2; sw = 0; ss = 2; break;     // the hybrid's over-the-cache form
    case 2: lw = 2; ls = 2; sw = 2; ss = 2; break;     // all non-temporal
    case 3: lw = 0; ls = 0; sw = 0; ss = 0; break;     // all plain
    case 4: lw = 0; ls = 2; sw = 16; ss = 16; break;   // nt state loads, write-through stores
    case 5: lw = 0; ls = 0; sw = 0; ss = 16; break;    // W plain, state write-through
    default: lw = 0; ls = 0; sw = 16; ss = 16; break;  // shipped (cache-resident state)
  }
}

template <bool ADAM, int FWDC, bool BF = false>
__global__ void __launch_bounds__(1024)
wgrad_group_kernel(WgGroup grp, int M, SlOpt o) {
  // FWDC: look-ahead row chunks of 16 (0 = no look-ahead; 1: next batch <= 16 rows; 4: <= 64)
  constexpr bool FWDN = FWDC > 0;
  __shared__ f32x4 sa[16][64];
  __shared__ float sdz[16][16];
  // look-ahead: the updated W tile, rows padded to 65 float4.
  // The MFMA B-layout read below takes 16 rows of one column: with a 1 KB row stride all
  // 16 hit the same LDS banks (rocprofv3 SQ_LDS_BANK_CONFLICT 3.96 M cycles per TP = 1
  // step, 0 without the look-ahead); one float4 of padding spreads them over all banks.
  __shared__ f32x4 sw[FWDN ? 16 * 65 : 1];
  __shared__ f32x4 red[FWDN ? 16 : 1][64];   // look-ahead: per-wave 16x16 partials
  // pick the layer with selects (no runtime-indexed access to the by-value argument)
  int bx, by;
  const int layer = wg_tile(grp, bx, by);
  const bool l0 = layer == 0;
  const WgDesc L = layer == 2 ? grp.d[2] : (l0 ? grp.d[0] : grp.d[1]);
  const int kb = bx * 256;
  if (kb >= L.K) return;                 // 2-D grid only; uniform per workgroup
  const int tid = threadIdx.x;
  const int r = tid >> 6, lane = tid & 63;
  const int n0 = by * 16;
  const int n = n0 + r;
  const int k = kb + lane * 4;
  const bool act = (n < L.N) && (k < L.K);
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  const int64_t off = (int64_t)n * L.ldw + k;
  // A / dZ of the first 16-row chunk ahead of W / m / v (grp.afirst, TP shards): a wave's
  // loads complete in order, so staged behind the state stream they held the LDS staging and
  // the dW product until W / m / v had arrived
  f32x4 av0 = zv;
  float dzv0 = 0.f;
  if (grp.afirst) {
    if (r < M && k < L.K) av0 = *reinterpret_cast<const f32x4*>(L.A + (int64_t)r * L.lda + k);
    if (tid < 256 && (tid >> 4) < M && n0 + (tid & 15) < L.N) dzv0 = L.dz[(int64_t)(tid >> 4) * L.ldz + n0 + (tid & 15)];
  }
  f32x4 p = zv, q0 = zv, q1 = zv;
  int plw = 0, pls = 0, psw = 16, pss = 16;
  pol_aux(grp.pol, plw, pls, psw, pss);
  const int lbytes = L.N * L.ldw * 4;   // grp.pol != 0 only for layers under 2 GB
  if (act) {
    if (grp.pol == 0) {
      p = *reinterpret_cast<const f32x4*>(L.W + off);
      q0 = *reinterpret_cast<const f32x4*>(L.s0 + off);
      if (ADAM) q1 = *reinterpret_cast<const f32x4*>(L.s1 + off);
    } else {
      p = ld_pol(L.W, lbytes, (int)(off * 4), plw);
      q0 = ld_pol(L.s0, lbytes, (int)(off * 4), pls);
      if (ADAM) q1 = ld_pol(L.s1, lbytes, (int)(off * 4), pls);
    }
  }
  // look-ahead A operand in MFMA layout: lane (li, lq) holds x_next[li][kb + 16*wave + 4*lq .. +3]
  const int li = lane & 15, lq = lane >> 4;
  const int kx = kb + 16 * r + 4 * lq;
  f32x4 xv[FWDC > 0 ? FWDC : 1];
#pragma unroll
  for (int c = 0; c < (FWDC > 0 ? FWDC : 1); ++c) {
    xv[c] = zv;
    if (FWDN && l0 && 16 * c + li < grp.mn && kx < L.K)
      xv[c] = *reinterpret_cast<const f32x4*>(grp.xn + (int64_t)(16 * c + li) * grp.ldxn + kx);
  }
  f32x4 g = zv;
  float gb = 0.f;
  f32x4 dacc = zv;   // bf16 form: dW[n0 + 4 lq + j][kb + 16 r + li] (MFMA accumulator layout)
  for (int mc = 0; mc < M; mc += 16) {
    if (mc) __syncthreads();
    {
      const int mm = mc + r;
      const bool pre = mc == 0 && grp.afirst;
      const f32x4 av = pre ? av0
                           : ((mm < M && k < L.K) ? *reinterpret_cast<const f32x4*>(L.A + (int64_t)mm * L.lda + k) : zv);
      sa[r][lane] = grp.bf16 ? bfr4(av) : av;
      if (tid < 256) {
        const int mr = mc + (tid >> 4), nn = n0 + (tid & 15);
        float v = 0.f;
        if (pre) v = dzv0;
        else if (mr < M && nn < L.N) v = L.dz[(int64_t)mr * L.ldz + nn];
        sdz[tid >> 4][tid & 15] = grp.bf16 ? bfr(v) : v;
      }
    }
    __syncthreads();
    if (BF) {
      // `--dtype bf16`: the tile's dW = dZ^T A on bf16 MFMA (v_mfma_f32_16x16x16_bf16, k = the
      // 16 batch rows of this chunk): wave r forms the 16 x 16 block of columns [16 r, 16 r + 16);
      // lane (li, lq) supplies dZ[4 lq .. 4 lq + 3][n0 + li] and A[4 lq .. 4 lq + 3][16 r + li]
      typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
      bf16x4_t av4, bv4;
      const int col = 16 * r + li;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        av4[t] = (__bf16)sdz[4 * lq + t][li];
        bv4[t] = (__bf16)sa[4 * lq + t][col >> 2][col & 3];
      }
      dacc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(av4, bv4, dacc, 0, 0, 0);
#pragma unroll
      for (int mm = 0; mm < 16; ++mm) gb += sdz[mm][r];
    } else {
#pragma unroll
      for (int mm = 0; mm < 16; ++mm) {
        const float d = sdz[mm][r];
        g += d * sa[mm][lane];
        gb += d;
      }
    }
  }
  if (BF) {
    // back to the update's layout (row r, float4 column lane) through the A tile's LDS
    __syncthreads();
    float* dws = reinterpret_cast<float*>(&sa[0][0]);   // [16][256]
#pragma unroll
    for (int j = 0; j < 4; ++j) dws[(4 * lq + j) * 256 + 16 * r + li] = dacc[j];
    __syncthreads();
    g = sa[r][lane];
  }
  if (act) {
    sl_opt_update4<ADAM>(o, p, g, q0, q1);
    if (grp.pol != 0) {
      const int boff = (int)(off * 4);
      if (o.kind != 0) st_pol(L.W, lbytes, boff, p, psw);
      st_pol(L.s0, lbytes, boff, q0, pss);
      if (ADAM) st_pol(L.s1, lbytes, boff, q1, pss);
    } else if (grp.wt) {
      const int boff = (int)(off * 4);
      if (o.kind != 0) st_wt(L.W, L.N, L.ldw, boff, p);
      st_wt(L.s0, L.N, L.ldw, boff, q0);
      if (ADAM) st_wt(L.s1, L.N, L.ldw, boff, q1);
    } else {
      if (o.kind != 0) *reinterpret_cast<f32x4*>(L.W + off) = p;
      *reinterpret_cast<f32x4*>(L.s0 + off) = q0;
      if (ADAM) *reinterpret_cast<f32x4*>(L.s1 + off) = q1;
    }
  }
  if (FWDN && l0) {
    // next batch's partial pre-activations with the updated tile: stage W_new through LDS
    // into MFMA B layout; wave w covers columns [16w, 16w+16) with 4 exact-fp32 MFMAs
    // (B[k][n] = W_new[n][k]: lane (n = li, k-group lq) reads one float4 of the tile)
    // rows padded to 65 float4 (a plain 64 and an XOR-swizzled layout measured the same)
    sw[r * 65 + lane] = act ? p : zv;
    __syncthreads();
    f32x4 wv4 = sw[li * 65 + 4 * r + lq];
    if (grp.bf16) wv4 = bfr4(wv4);
#pragma unroll
    for (int c = 0; c < FWDC; ++c) {
      if (16 * c >= grp.mn) break;        // uniform
      f32x4 z = zv;
      const f32x4 xc = grp.bf16 ? bfr4(xv[c]) : xv[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) z = __builtin_amdgcn_mfma_f32_16x16x4f32(xc[i], wv4[i], z, 0, 0, 0);
      if (c) __syncthreads();             // the previous chunk's readers are done with red
      red[r][lane] = z;                   // z[j] = partial(m = 16c + 4*lq + j, n = n0 + li)
      __syncthreads();
      if (tid < 256) {
        const int m = 16 * c + (tid >> 4), nn = tid & 15;
        const int mm = tid >> 4;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 16; ++w) v += red[w][16 * (mm >> 2) + nn][mm & 3];
        if (m < grp.mn && n0 + nn < L.N) grp.pn[((int64_t)bx * grp.mn + m) * L.N + n0 + nn] = v;
      }
    }
  }
  if (L.bias && bx == 0 && lane == 0 && n < L.N) {
    float pb = L.bias[n], b0 = L.sb0[n], b1 = L.sb1 ? L.sb1[n] : 0.f;
    sl_opt_update(o, pb, gb, b0, b1);
    if (o.kind != 0) L.bias[n] = pb;
    L.sb0[n] = b0;
    if (L.sb1) L.sb1[n] = b1;
  }
}

// wgrad_stream_kernel: wgrad_group_kernel's fp32 update (M <= 16 rows, look-ahead of <= 16 rows)
// as a column walk: workgroup = (layer, 256-column block bx, a run of grp.rt consecutive 16-row
// tiles).  The tiled form stages A (and the look-ahead's x) once per 16 x 256 tile and holds one
// tile's W / m / v per thread, so a CU's in-flight bytes drop to nothing while a workgroup
// stages, sums and stores; over concat's 2.6 GB fc1 state it streams at 4.4-4.7 TB/s
// (profiles/r5w_misc/wgbench_split_concat_policy.txt).  Here A and x are staged once per run,
// each wave takes its row's 16 dZ values in lanes 0-15 (read back with v_readlane: no LDS
// staging, no barrier per tile without the look-ahead), and the next tile's W / m / v / dZ loads
// are issued before the current tile's update, so every thread keeps a tile's state in flight
// across the whole run.  Every element's sums are the tiled form's, in its order: bitwise equal.
template <bool ADAM, bool FWDN>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
wgrad_stream_kernel(WgGroup grp, int M, SlOpt o) {
  __shared__ f32x4 sa[16][64];
  __shared__ f32x4 sw[FWDN ? 16 * 65 : 1];
  __shared__ f32x4 red[FWDN ? 16 : 1][64];
  const int lin = (int)blockIdx.x;
  const int li = (grp.n > 2 && lin >= grp.d[2].wb0) ? 2 : ((grp.n > 1 && lin >= grp.d[1].wb0) ? 1 : 0);
  const int wb0 = li == 2 ? grp.d[2].wb0 : (li == 1 ? grp.d[1].wb0 : 0);
  const bool l0 = li == 0;
  const WgDesc L = li == 2 ? grp.d[2] : (l0 ? grp.d[0] : grp.d[1]);
  const int kx = (L.K + 255) >> 8;
  int local = lin - wb0;
  if (l0 && grp.rev0) local = grp.nt0 - 1 - local;
  const int byg = __builtin_amdgcn_readfirstlane(local / kx);
  const int bx = local - byg * kx;
  const int kb = bx * 256;
  const int ny = (L.N + 15) >> 4;
  const int t0 = byg * grp.rt, t1 = min(ny, t0 + grp.rt);
  const int tid = threadIdx.x;
  const int r = tid >> 6, lane = tid & 63;
  const int k = kb + lane * 4;
  const bool kin = k < L.K;
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  int plw = 0, pls = 0, psw = 16, pss = 16;
  // with layer 0 pinned, the small layers (concat's fc2 / fc3, 70 MB) keep the over-the-cache
  // form (W plain, m / v non-temporal): W2 / W3 are read again by the next kernels (fc2 forward
  // 10.7 -> 8 us per concat step with W2 in the Infinity Cache)
  pol_aux(l0 || grp.pin == 0 ? grp.pol : 1, plw, pls, psw, pss);
  const int lbytes = L.N * L.ldw * 4;   // grp.pol != 0 only for layers under 2 GB
  // one tile's state for this thread: W / m / v of (row 16 by + r, columns k .. k + 3), and the
  // wave's dZ[lane][16 by + r] in lanes 0-15
  // a pinned tile (layer 0, rows < grp.pin): plain both ways
  const auto pinned = [&](int by) { return l0 && by * 16 < grp.pin; };
  auto ld_tile = [&](int by, f32x4& p, f32x4& q0, f32x4& q1, float& dzl) {
    const int n = by * 16 + r;
    dzl = (lane < 16 && lane < M && n < L.N) ? L.dz[(int64_t)lane * L.ldz + n] : 0.f;
    p = zv;
    q0 = zv;
    q1 = zv;
    if (n < L.N && kin) {
      const int64_t off = (int64_t)n * L.ldw + k;
      if (grp.pol == 0) {
        p = *reinterpret_cast<const f32x4*>(L.W + off);
        q0 = *reinterpret_cast<const f32x4*>(L.s0 + off);
        if (ADAM) q1 = *reinterpret_cast<const f32x4*>(L.s1 + off);
      } else {
        const bool pn = pinned(by);
        p = ld_pol(L.W, lbytes, (int)(off * 4), pn ? 0 : plw);
        q0 = ld_pol(L.s0, lbytes, (int)(off * 4), pn ? 0 : pls);
        if (ADAM) q1 = ld_pol(L.s1, lbytes, (int)(off * 4), pn ? 0 : pls);
      }
    }
  };
  f32x4 p, q0, q1;
  float dzl;
  ld_tile(t0, p, q0, q1, dzl);
  // A rows (zero past M) and the look-ahead's x (MFMA A layout, lane (li, lq): x_next[li][kb +
  // 16 wave + 4 lq ..]) of this column block, once for the whole run
  const int xi = lane & 15, xq = lane >> 4;
  const int kxn = kb + 16 * r + 4 * xq;
  f32x4 xv = zv;
  if (FWDN && l0 && xi < grp.mn && kxn < L.K) xv = *reinterpret_cast<const f32x4*>(grp.xn + (int64_t)xi * grp.ldxn + kxn);
  sa[r][lane] = (r < M && kin) ? *reinterpret_cast<const f32x4*>(L.A + (int64_t)r * L.lda + k) : zv;
  __syncthreads();
  for (int by = t0; by < t1; ++by) {
    f32x4 pn_ = zv, qn0 = zv, qn1 = zv;
    float dzn = 0.f;
    if (by + 1 < t1) ld_tile(by + 1, pn_, qn0, qn1, dzn);   // uniform
    const int n0 = by * 16, n = n0 + r;
    const bool act = n < L.N && kin;
    f32x4 g = zv;
    float gb = 0.f;
    // (fully unrolled the form without the look-ahead hoists all 16 LDS reads and spills at
    // 8 waves per SIMD; unrolled by 4 the look-ahead form spills instead)
    if constexpr (FWDN) {
#pragma unroll
      for (int mm = 0; mm < 16; ++mm) {
        const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, dzl), mm));
        g += d * sa[mm][lane];
        gb += d;
      }
    } else {
#pragma unroll 4
      for (int mm = 0; mm < 16; ++mm) {
        const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, dzl), mm));
        g += d * sa[mm][lane];
        gb += d;
      }
    }
    if (act) {
      sl_opt_update4<ADAM>(o, p, g, q0, q1);
      const int64_t off = (int64_t)n * L.ldw + k;
      if (grp.pol != 0) {
        const int boff = (int)(off * 4);
        const bool pn = pinned(by);
        if (o.kind != 0) st_pol(L.W, lbytes, boff, p, pn ? 0 : psw);
        st_pol(L.s0, lbytes, boff, q0, pn ? 0 : pss);
        if (ADAM) st_pol(L.s1, lbytes, boff, q1, pn ? 0 : pss);
      } else if (grp.wt) {
        const int boff = (int)(off * 4);
        if (o.kind != 0) st_wt(L.W, L.N, L.ldw, boff, p);
        st_wt(L.s0, L.N, L.ldw, boff, q0);
        if (ADAM) st_wt(L.s1, L.N, L.ldw, boff, q1);
      } else {
        if (o.kind != 0) *reinterpret_cast<f32x4*>(L.W + off) = p;
        *reinterpret_cast<f32x4*>(L.s0 + off) = q0;
        if (ADAM) *reinterpret_cast<f32x4*>(L.s1 + off) = q1;
      }
    }
    if (FWDN && l0) {
      // the tiled form's look-ahead, tile by tile (sw / red reuse: the barrier after red's
      // writes follows every read of sw, the next tile's first barrier every read of red)
      sw[r * 65 + lane] = act ? p : zv;
      __syncthreads();
      const f32x4 wv4 = sw[xi * 65 + 4 * r + xq];
      f32x4 z = zv;
#pragma unroll
      for (int i = 0; i < 4; ++i) z = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[i], wv4[i], z, 0, 0, 0);
      red[r][lane] = z;
      __syncthreads();
      if (tid < 256) {
        const int m = tid >> 4, nn = tid & 15;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 16; ++w) v += red[w][16 * (m >> 2) + nn][m & 3];
        if (m < grp.mn && n0 + nn < L.N) grp.pn[((int64_t)bx * grp.mn + m) * L.N + n0 + nn] = v;
      }
    }
    if (L.bias && bx == 0 && lane == 0 && n < L.N) {
      float pb = L.bias[n], b0 = L.sb0[n], b1 = L.sb1 ? L.sb1[n] : 0.f;
      sl_opt_update(o, pb, gb, b0, b1);
      if (o.kind != 0) L.bias[n] = pb;
      L.sb0[n] = b0;
      if (L.sb1) L.sb1[n] = b1;
    }
    p = pn_;
    q0 = qn0;
    q1 = qn1;
    dzl = dzn;
  }
}

int head3_slices(int N2) { return max(1, (N2 / 4 + HS - 1) / HS); }

static dim3 head_grid(int M, int Q) { return dim3(Q, M); }

static void launch_head_bwd(const float* plog, const float* b3, const float* W3, int ldw3, const int64_t* y,
                            int64_t ignore, float scale, float dscale, const float* h2, float* dlog, float* dz2,
                            float* loss_rows, int M, int N2, int C, int Q, int Qp, hipStream_t st, int G,
                            const float* gscale) {
  const size_t sh = (size_t)C * sizeof(float);
  const dim3 g = head_grid(M, Q);
  if (g_bf16)
    head_bwd_kernel<true><<<g, 256, sh, st>>>(plog, b3, W3, ldw3, y, ignore, scale, dscale, h2, dlog, dz2, loss_rows,
                                              M, N2, C, Qp, G, gscale);
  else
    head_bwd_kernel<false><<<g, 256, sh, st>>>(plog, b3, W3, ldw3, y, ignore, scale, dscale, h2, dlog, dz2,
                                               loss_rows, M, N2, C, Qp, G, gscale);
}

hipError_t server_head3(const float* P2, int S2, int64_t slab2, Epi e2, const float* W3, int ldw3, const float* b3,
                        const int64_t* y, int64_t ignore, float scale, float* h2, float* dlog, float* dz2,
                        float* loss_rows, float* ws, int64_t ws_elems, int M, int N2, int C, hipStream_t st,
                        const IpcStep* ipc, int G, const float* gscale) {
  if (M <= 0) return hipSuccess;
  if ((N2 & 3) || (ldw3 & 3) || G < 1 || C % G != 0) return hipErrorInvalidValue;
  const int Q = head3_slices(N2);
  if (ws_elems < (int64_t)Q * M * C) return hipErrorInvalidValue;
  const dim3 g = head_grid(M, Q);
  if (ipc != nullptr && (S2 < 1 || (slab2 & 3) || (int64_t)M * Q > ipc->nflags || (int64_t)M * N2 > ipc->cap ||
                         ipc->T < 1 || ipc->T > kIpcMaxRanks))
    return hipErrorInvalidValue;
  const IpcStep none{};
  const IpcStep& ip = ipc ? *ipc : none;
  // a wide head's output groups (104 logits each) spread over gridDim.z: C = 800 (SISA-concat,
  // k = 8) ran 128 workgroups of 8 groups each
  dim3 gf = g;
  if (ipc == nullptr) gf.z = (unsigned)std::max(1, std::min(8, (C + 103) / 104));
  if (ipc != nullptr) {
    if (g_bf16)
      head_fwd_kernel<true, true><<<g, 256, 0, st>>>(P2, S2, slab2, e2, W3, ldw3, h2, ws, M, N2, C, ip);
    else
      head_fwd_kernel<false, true><<<g, 256, 0, st>>>(P2, S2, slab2, e2, W3, ldw3, h2, ws, M, N2, C, ip);
  } else {
    if (g_bf16)
      head_fwd_kernel<true, false><<<gf, 256, 0, st>>>(P2, S2, slab2, e2, W3, ldw3, h2, ws, M, N2, C, none);
    else
      head_fwd_kernel<false, false><<<gf, 256, 0, st>>>(P2, S2, slab2, e2, W3, ldw3, h2, ws, M, N2, C, none);
  }
  launch_head_bwd(ws, b3, W3, ldw3, y, ignore, scale, e2.dscale, h2, dlog, dz2, loss_rows, M, N2, C, Q, Q, st, G,
                  gscale);
  return hipGetLastError();
}

// Per-launch traversal / store form.  The direction of layer 0's walk alternates from one
// launch to the next (graph capture bakes the pattern in; every captured chunk has an even
// number of steps).  W/m/v are stored write-through (32-bit byte offsets: layers under 2 GB
// only; plain stores otherwise).  Measured (scripts/cache_ab.py, one process, interleaved
// rounds, us per look-ahead server step at TP = 1 / 2 / 4 / 8): always-forward 183.4 /
// 102.2 / 70.2 / 59.7, alternating 172.6 / 100.9 / 69.6 / 59.8, alternating +
// write-through 171.8 / 100.9 / 68.7 / 59.5 (profiles/r1_cache_ab.txt).
static void set_traversal(WgGroup& gg) {
  static unsigned flip = 0;
  gg.rev0 = (int)(flip++ & 1u);
  gg.wt = 1;
  gg.bf16 = g_bf16;
  for (int i = 0; i < gg.n; ++i)
    if ((int64_t)gg.d[i].N * gg.d[i].ldw * 4 > 2147483647LL) gg.wt = 0;
  // a layer-0 stream larger than the 256 MB Infinity Cache (concat's fc1, SISA's TP = 1 fc1 on
  // launch-per-stage) takes the hybrid's over-the-cache policy: W plain both ways (it stays
  // cached from one step to the next), the optimizer state non-temporal both ways.  ws = 9
  // concat on one GPU 88.1-88.4 k -> 90.0 k; vanilla and U-shape, whose state fits, are
  // fastest as shipped (profiles/r5w_misc/wgrad_group_cache_policy_ab.txt).  Variant 21 forces
  // a preset (pol_aux; 6 = the shipped one).
  const int64_t st0 = (int64_t)gg.d[0].N * gg.d[0].ldw * 4 * (gg.d[0].s1 ? 3 : 2);
  const int v21 = g_variant[21];
  gg.pol = !gg.wt ? 0 : (v21 == 6 ? 0 : (v21 != 0 ? v21 : (st0 > (256ll << 20) ? 1 : 0)));
  // A layer-0 stream of over 1 GB (concat's fc1: 2.6 GB of W / m / v, 519 KB per row) instead
  // pins a fixed subset of its rows in the Infinity Cache -- plain loads and stores of their W /
  // m / v, ~65 % of the 256 MB, so those rows never reach HBM -- and streams every other row
  // non-temporal past it.  ws = 9 concat on one GPU (profiles/r6_pin/): 92.5 -> 96.4-97.6 k on one
  // box, 320 rows the best of 192 - 576 on another.  Variant 23 forces a row count (-1: off).
  gg.pin = 0;
  const int64_t row0 = (int64_t)gg.d[0].ldw * 4 * (gg.d[0].s1 ? 3 : 2);
  const int v23 = g_variant[23];
  if (gg.wt && v23 >= 0) {
    int pin = v23 > 0 ? v23 : (st0 > (1ll << 30) ? (int)((256ll << 20) * 65 / 100 / row0) : 0);
    pin = pin / 16 * 16;
    if (pin > 0) {
      gg.pin = pin;
      gg.pol = 2;
    }
  }
}

hipError_t wgrad_group(const WgGroup& g, int M, SlOpt o, hipStream_t st) {
  int kmax = 0, yb = 0, wb = 0;
  WgGroup gg = g;
  set_traversal(gg);
  for (int i = 0; i < gg.n; ++i) {
    if (gg.d[i].dz == nullptr) return hipErrorInvalidValue;
    gg.d[i].yb0 = yb;
    gg.d[i].wb0 = wb;
    yb += (gg.d[i].N + 15) / 16;
    wb += ((gg.d[i].N + 15) / 16) * ((gg.d[i].K + 255) / 256);
    kmax = max(kmax, gg.d[i].K);
  }
  if (yb == 0 || kmax == 0) return hipSuccess;
  gg.nt0 = ((gg.d[0].N + 15) / 16) * ((gg.d[0].K + 255) / 256);
  const dim3 grid((kmax + 255) / 256, yb);   // 2-D: (K blocks of the widest layer) x (row tiles)
  const dim3 grid1(wb);                      // 1-D over the real tiles
  if (gg.xn && (gg.mn <= 0 || gg.mn > 64 || !gg.pn)) return hipErrorInvalidValue;
  const bool fw = gg.xn != nullptr;
  const int fc = (fw && gg.mn > 16) ? 4 : (fw ? 1 : 0);
  // The streaming form for fp32 steps of <= 16 rows: runs of 4 row tiles from 8,000 tiles
  // (>= 2,000 workgroups), of 2 from 1,280, else the tiled form.  wgbench (us per call, tiled ->
  // stream; profiles/r6_wg/): concat's fc1 + fc2 + fc3 1,149 -> 1,002 (rt 4: 4.6 -> 5.3 TB/s of
  // state), vanilla's 112 -> 92 (rt 4), the SISA tail at TP = 1 / 2 / 4 151 / 66.5 / 37.4 -> 137 /
  // 62.9 / 36.7 (rt 4 / 2 / 2; rt 4 at TP = 2: 68), U-shape's 30.1 -> 27.5 (rt 2); a TP = 8 shard
  // (1,097 tiles) keeps the tiled form (22.2 against 23.8 at rt 2).  Variant 22: -1 forces the
  // tiled form, > 0 forces that run length.
  int rt = g_variant[22];
  if (rt == 0) {
    int tiles = 0;
    for (int i = 0; i < gg.n; ++i) tiles += ((gg.d[i].K + 255) / 256) * ((gg.d[i].N + 15) / 16);
    rt = tiles >= 8000 ? 4 : (tiles >= 1280 ? 2 : 0);
  }
  if (rt > 0 && !gg.bf16 && M <= 16 && fc <= 1) {
    WgGroup gs = gg;
    gs.rt = rt;
    int ws = 0;
    for (int i = 0; i < gs.n; ++i) {
      gs.d[i].wb0 = ws;
      ws += ((gs.d[i].K + 255) / 256) * (((gs.d[i].N + 15) / 16 + rt - 1) / rt);
      if (i == 0) gs.nt0 = ws;
    }
    if (o.kind == 2) {
      if (fw) wgrad_stream_kernel<true, true><<<ws, 1024, 0, st>>>(gs, M, o);
      else wgrad_stream_kernel<true, false><<<ws, 1024, 0, st>>>(gs, M, o);
    } else {
      if (fw) wgrad_stream_kernel<false, true><<<ws, 1024, 0, st>>>(gs, M, o);
      else wgrad_stream_kernel<false, false><<<ws, 1024, 0, st>>>(gs, M, o);
    }
    return hipGetLastError();
  }
  // 2-D grid when it wastes < 10 % of its workgroups (TP = 1: 3 %, measured 1.4 us per step
  // faster there), else the 1-D grid (TP = 2 / 4 / 8: 18-55 % empty, 0.3-1.2 us faster;
  // profiles/r1_cache_ab_grid.txt)
  const int64_t g2 = (int64_t)grid.x * grid.y;
  gg.grid2d = (g2 - wb) * 10 < g2 ? 1 : 0;
  const dim3 gr = gg.grid2d ? grid : grid1;
  // the first chunk's A / dZ loads ahead of W / m / v on a TP shard (1-D grid), whose state
  // streams from the Infinity Cache: native executor, us per server step, TP = 4 68.8 -> 66.2,
  // TP = 8 52.5 -> 51.2; at TP = 1 (2-D grid, HBM-bound) 170.9 vs 171.2, so not there
  // (profiles/r3w_wgrad_a_first_ab.txt)
  gg.afirst = gg.grid2d ? 0 : 1;
  // bf16 compute: a separate instantiation (dW on bf16 MFMA), so the fp32 kernels' registers
  // and schedule are untouched
#define SL_WG_LAUNCH(A, F)                                                          \
  do {                                                                              \
    if (gg.bf16) wgrad_group_kernel<A, F, true><<<gr, 1024, 0, st>>>(gg, M, o);      \
    else wgrad_group_kernel<A, F, false><<<gr, 1024, 0, st>>>(gg, M, o);            \
  } while (0)
  if (o.kind == 2) {
    if (fc == 4) SL_WG_LAUNCH(true, 4);
    else if (fc) SL_WG_LAUNCH(true, 1);
    else SL_WG_LAUNCH(true, 0);
  } else {
    if (fc == 4) SL_WG_LAUNCH(false, 4);
    else if (fc) SL_WG_LAUNCH(false, 1);
    else SL_WG_LAUNCH(false, 0);
  }
#undef SL_WG_LAUNCH
  return hipGetLastError();
}

}  // namespace sl
