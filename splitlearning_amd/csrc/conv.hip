// Client-front kernels: fused gather + conv3x3(1->32) + bias + ReLU + maxpool2x2
// forward, and fused pool/ReLU backward + weight/bias gradient + optimizer step.
//
// Reference ops: models.py:8-9,21-23 (Conv2d(1,32,3) -> ReLU -> MaxPool(2,2)),
// trained with Adam(wd=1e-5) (data_entities_vanilla_sisa.py:48) or SGD-m via the
// DistributedOptimizer (data_entities_vanilla.py:37-42).  SURVEY §2.7 K1-K3, K13.
//
// The conv has K = 9 (one input channel), far too small for MFMA, so it is a
// direct LDS-tiled convolution: a 256-thread workgroup per (sample, 8 output channels)
// stages the 28x28 image (converted from the uint8 shard row it gathers itself, so there
// is no separate collate/convert kernel) and its 8x9 weights in LDS and writes its part of
// the pooled, NCHW-flattened [5408] activation plus a 2-bit argmax for backward.
#include "common.h"

#include <algorithm>
#include <vector>

namespace sl {

// One pooled output: 4x4 input patch -> 2x2 conv outputs -> bias, max (first max, torch
// order), ReLU; `arg` is the 2-bit position of the max for the backward.
// The 28 x 28 image in LDS, split by column parity: column c of row r sits at
// (c & 1) * IMG_PLANE + r * IMG_RS + (c >> 1).  Lanes own consecutive pooled columns pw, so
// a plain row-major image has them read columns 2 pw + j (stride 2: 2-way bank conflicts,
// 34-45 % of the conv kernels' LDS cycles in an SQ counter pass, profiles/r1_pmc_bench_lds.txt);
// here each read is consecutive words within a plane, and the 39-word row stride (78 = 14
// mod 64 banks per pooled row) keeps the ~5 pooled rows of a wave on distinct banks.
constexpr int IMG_RS = 39, IMG_PLANE = 28 * IMG_RS, IMG_LDS = 2 * IMG_PLANE;
__device__ __forceinline__ int img_idx(int r, int c) { return (c & 1) * IMG_PLANE + r * IMG_RS + (c >> 1); }

__device__ __forceinline__ void conv_pool_at(const float* img, const float* wk, float bias, int ph, int pw,
                                             float& y, int& arg) {
  const float* base = img + (2 * ph) * IMG_RS + pw;
  float patch[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) patch[i][j] = base[(j & 1) * IMG_PLANE + i * IMG_RS + (j >> 1)];
  float best = 0.f;
  arg = 0;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      float acc = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) acc = fmaf(wk[kh * 3 + kw], patch[dy + kh][dx + kw], acc);
      acc += bias;
      const int pos = dy * 2 + dx;
      if (pos == 0 || acc > best) { best = acc; arg = pos; }
    }
  y = fmaxf(best, 0.f);
}

// Deferred client optimizer step (split modes, FrontEngine): parameter slot p (slab layout
// oc*10 + j; j = 9 is the bias) updated from the previous backward's pB partial slabs with
// exactly conv_opt_reduce_kernel's arithmetic.  Returns the new value, a0/a1 the new states.
__device__ __forceinline__ float conv_pending_param(const float* w, const float* b, const float* s0w,
                                                   const float* s1w, const float* s0b, const float* s1b,
                                                   const float* pslab, int pB, int p, const SlOpt& o,
                                                   float& a0, float& a1) {
  const int oc = p / 10, j = p - oc * 10;
  const bool isw = j < 9;
  const int k = isw ? oc * 9 + j : oc;
  float pp = isw ? w[k] : b[k];
  a0 = isw ? s0w[k] : s0b[k];
  a1 = isw ? (s1w ? s1w[k] : 0.f) : (s1b ? s1b[k] : 0.f);
  const float g = sum_slabs(pslab + p, pB, 320);
  sl_opt_update(o, pp, g, a0, a1);
  return pp;
}

// Grid (B, 4): workgroup (s, q) computes channels [8q, 8q + 8) of sample s (1352 pooled
// outputs, 5-6 per thread), so a batch of 16 runs 64 workgroups instead of 16 and each
// thread's serial chain is a quarter as long (the per-sample 256-thread form measured
// 11 us per batch of 16 in the split modes, where this kernel is on the critical path).
// One (sample s = shard row src, channel group q) of the forward; am == nullptr: no argmax
// (frozen-front forwards: evaluation, activation dumps).
template <typename XT>
__device__ __forceinline__ void conv_fwd_sample(const XT* __restrict__ x, int64_t src, int s, int q,
                                                const float* __restrict__ w, const float* __restrict__ b,
                                                float* __restrict__ y, uint8_t* __restrict__ am,
                                                const int64_t* __restrict__ lab_in, int64_t* __restrict__ lab_out,
                                                const float* __restrict__ pslab, int pB, const float* __restrict__ s0w,
                                                const float* __restrict__ s1w, const float* __restrict__ s0b,
                                                const float* __restrict__ s1b, const SlOpt& o) {
  constexpr int CH = 8, NO = CH * 169, PER = (NO + 255) / 256;
  __shared__ float img[IMG_LDS];
  __shared__ float sw[CH * 9];
  __shared__ float sb[CH];
  const int tid = threadIdx.x;
  // every independent load goes out before anything is consumed
  const XT* xr = x + src * 784;
  const float p0 = (float)xr[tid], p1 = (float)xr[256 + tid], p2 = (float)xr[512 + tid];
  const float p3 = tid < 784 - 768 ? (float)xr[768 + tid] : 0.f;
  if (lab_in && q == 0 && tid == 0) lab_out[s] = lab_in[src];     // the batch's labels, gathered in passing
  if (pslab) {
    // the previous backward's optimizer step, applied here for this group's 8 channels
    // (80 parameters); FrontEngine's next backward stores the same values
    if (tid < CH * 10) {
      float a0, a1;
      const float pp = conv_pending_param(w, b, s0w, s1w, s0b, s1b, pslab, pB, q * CH * 10 + tid, o, a0, a1);
      const int c = tid / 10, j = tid - c * 10;
      if (j < 9) sw[c * 9 + j] = pp; else sb[c] = pp;
    }
  } else {
    const float wv = tid < CH * 9 ? w[q * CH * 9 + tid] : 0.f;
    const float bv = tid < CH ? b[q * CH + tid] : 0.f;
    if (tid < CH * 9) sw[tid] = wv;
    if (tid < CH) sb[tid] = bv;
  }
  img[img_idx(tid / 28, tid % 28)] = p0;
  img[img_idx((256 + tid) / 28, (256 + tid) % 28)] = p1;
  img[img_idx((512 + tid) / 28, (512 + tid) % 28)] = p2;
  if (tid < 784 - 768) img[img_idx((768 + tid) / 28, (768 + tid) % 28)] = p3;
  __syncthreads();
  float* yo = y + (int64_t)s * 5408 + q * NO;
  uint8_t* ao = am ? am + (int64_t)s * 5408 + q * NO : nullptr;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int o = tid + 256 * u;
    if (o < NO) {
      const int oc = o / 169;
      const int r = o - oc * 169;
      const int ph = r / 13;
      const int pw = r - ph * 13;
      float yv;
      int arg;
      conv_pool_at(img, sw + oc * 9, sb[oc], ph, pw, yv, arg);
      yo[o] = yv;
      if (ao) ao[o] = (uint8_t)arg;
    }
  }
}

template <typename XT>
__global__ void __launch_bounds__(256)
conv_relu_pool_fwd_kernel(const XT* __restrict__ x, const int64_t* __restrict__ idx, int64_t row0,
                          const float* __restrict__ w, const float* __restrict__ b,
                          float* __restrict__ y, uint8_t* __restrict__ am,
                          const int64_t* __restrict__ lab_in = nullptr, int64_t* __restrict__ lab_out = nullptr,
                          const float* __restrict__ pslab = nullptr, int pB = 0, const float* __restrict__ s0w = nullptr,
                          const float* __restrict__ s1w = nullptr, const float* __restrict__ s0b = nullptr,
                          const float* __restrict__ s1b = nullptr, SlOpt o = SlOpt{}) {
  const int s = blockIdx.x;
  conv_fwd_sample<XT>(x, idx ? idx[s] : row0 + s, s, (int)blockIdx.y, w, b, y, am, lab_in, lab_out, pslab, pB, s0w,
                      s1w, s0b, s1b, o);
}

// Frozen-front forward of several co-located Alices in one launch (evaluation and the SISA
// activation dump, reference data_entities_vanilla_sisa.py:196-211,370-371): grid (rows,
// 4, Alices); Alice a's rows [r0, r0 + gridDim.x) of her order, clipped to her n.  No argmax.
__global__ void __launch_bounds__(256) conv_fwd_multi_kernel(FrontFwdSet set, int64_t r0) {
  const FrontFwdDesc& d = set.d[blockIdx.z];
  const int64_t r = r0 + blockIdx.x;
  if (r >= d.n) return;                  // uniform per workgroup
  conv_fwd_sample<uint8_t>(d.x, d.idx ? d.idx[r] : r, (int)r, (int)blockIdx.y, d.w, d.b, d.y, nullptr, nullptr,
                           nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, SlOpt{});
}

// ---------------------------------------------------------------------------------------
// Two-stage backward + optimizer (a first single-kernel version, 32 workgroups each reducing
// one channel over the whole batch, left most of the GPU idle):
//   stage 1, one workgroup per sample: thread t owns output channel t>>3 and every 8th
//   pooled position of it, so its dW/db contributions all go to ONE channel and are
//   reduced by three xor-shuffles inside 8-lane groups -> slab[s][oc*10 + j];
//   stage 2, one workgroup: sum the B slabs and apply SGD-m / Adam to the 320 params.
// The SISA local step fuses stage 1 with the forward and the 5408-way softmax-CE of the
// activation (Q5): the activation never leaves registers.

__device__ __forceinline__ void conv_acc_grad(const float* img, int ph, int pw, int a, float g, float* acc) {
  const int r0 = 2 * ph + (a >> 1), c0 = 2 * pw + (a & 1);
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] = fmaf(g, img[img_idx(r0 + kh, c0 + kw)], acc[kh * 3 + kw]);
  acc[9] += g;
}

// Sum the 10 per-thread partials over the SUB consecutive lanes that share a channel.
template <int SUB>
__device__ __forceinline__ void slab_write(float* acc, float* dst, int sub) {
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    acc[j] = sl_group_sum<SUB>(acc[j]);
  }
  if (sub == 0) {
#pragma unroll
    for (int j = 0; j < 10; ++j) dst[j] = acc[j];
  }
}


template <typename XT>
__device__ __forceinline__ void stage_sample(const XT* x, int64_t src, const float* w, const float* b, float* img,
                                             float* sw, float* sb) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const XT* xr = x + src * 784;
  for (int i = tid; i < 784; i += nt) img[img_idx(i / 28, i % 28)] = (float)xr[i];
  for (int i = tid; i < 288; i += nt) sw[i] = w[i];
  if (tid < 32) sb[tid] = b[tid];
  __syncthreads();
}

// SISA local step, stage 1: forward + softmax-CE over the 5408-wide activation + dW/db
// partials, one workgroup per sample.  SUB lanes share an output channel (channel =
// tid / SUB), each owning every SUB-th of its 169 pooled positions.  At batch 16 only 16
// workgroups run, so the step is latency-bound: SUB = 32 (1024 threads, 6 positions per
// thread) cuts each thread's serial conv/CE/grad chain ~4x against SUB = 8 (22 per thread).
//
// FUSE (the epoch loop): the previous step's optimizer update is folded into this step's
// prologue instead of a separate 1-workgroup launch per step.  Every workgroup sums the
// previous step's B slabs and applies SGD-m / Adam to the 320 parameters of buffer `pin`
// (identical arithmetic to conv_opt_reduce_kernel), keeps the result in LDS for its own
// forward, and workgroup 0 also stores it to `pout` (ping-pong: no workgroup reads what
// another is writing).  Param buffer layout: [w 288 | b 32 | s0 320 | s1 320].
template <typename XT, int SUB, bool FUSE>
__device__ __forceinline__ void
conv_step_body(const XT* __restrict__ x, const int64_t* __restrict__ idx, const int64_t* __restrict__ labels,
               const float* __restrict__ w, const float* __restrict__ b, float scale, float* __restrict__ slab,
               float* __restrict__ loss_rows, const float* __restrict__ prev_slab, int Bprev,
               float* __restrict__ pout, SlOpt o, const int s) {
  constexpr int NJ = (169 + SUB - 1) / SUB;
  constexpr int NW = 32 * SUB / 64;
  __shared__ float img[IMG_LDS];
  __shared__ float sw[32 * 9];
  __shared__ float sb[32];
  __shared__ float red[2 * NW];
  const int tid = threadIdx.x;
  const int64_t src = idx[s];
  // every load that does not depend on another goes out before anything is consumed: the
  // sample's label and pixels, and (FUSE) the previous step's B slabs and parameters —
  // one memory round trip after the index instead of one per slab
  const int64_t lab = labels[src];
  if (FUSE && 32 * SUB >= 784) {
    const XT* xr = x + src * 784;
    const float px = tid < 784 ? (float)xr[tid] : 0.f;
    const float* pin = w;      // [w | b | s0 | s1] of the previous step
    if (tid < 320) {
      const int p = tid, oc = p / 10, j = p - (p / 10) * 10;
      const int k = j < 9 ? oc * 9 + j : 288 + oc;
      float pp = pin[k], a0 = pin[320 + k], a1 = pin[640 + k];
      if (prev_slab) {
        const float g = sum_slabs(prev_slab + p, Bprev, 320);
        sl_opt_update(o, pp, g, a0, a1);
        if (s == 0) {
          pout[k] = pp;
          pout[320 + k] = a0;
          pout[640 + k] = a1;
        }
      }
      if (k < 288) sw[k] = pp; else sb[k - 288] = pp;
    }
    if (tid < 784) img[img_idx(tid / 28, tid % 28)] = px;
    __syncthreads();
  } else if (FUSE) {
    const float* pin = w;
    for (int p = tid; p < 320; p += 32 * SUB) {
      const int oc = p / 10, j = p - (p / 10) * 10;
      const int k = j < 9 ? oc * 9 + j : 288 + oc;
      float pp = pin[k], a0 = pin[320 + k], a1 = pin[640 + k];
      if (prev_slab) {
        const float g = sum_slabs(prev_slab + p, Bprev, 320);
        sl_opt_update(o, pp, g, a0, a1);
        if (s == 0) {
          pout[k] = pp;
          pout[320 + k] = a0;
          pout[640 + k] = a1;
        }
      }
      if (k < 288) sw[k] = pp; else sb[k - 288] = pp;
    }
    const XT* xr = x + src * 784;
    for (int i = tid; i < 784; i += 32 * SUB) img[img_idx(i / 28, i % 28)] = (float)xr[i];
    __syncthreads();
  } else {
    stage_sample(x, src, w, b, img, sw, sb);
  }
  const int oc = tid / SUB, sub = tid % SUB;
  const float* wk = sw + oc * 9;
  const float bias = sb[oc];
  float yv[NJ];
  int av[NJ];
  float mx = 0.f;   // activations are >= 0 after ReLU
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int r = sub + SUB * j;
    yv[j] = -1.f;
    av[j] = 0;
    if (r < 169) {
      const int ph = r / 13, pw = r - (r / 13) * 13;
      conv_pool_at(img, wk, bias, ph, pw, yv[j], av[j]);
      mx = fmaxf(mx, yv[j]);
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
  mx = sl_wave_max(mx);
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) mx = fmaxf(mx, red[i]);
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    if (sub + SUB * j < 169) se += expf(yv[j] - mx);
  se = sl_wave_sum(se);
  if (lane == 0) red[NW + wv] = se;
  __syncthreads();
  se = red[NW];
#pragma unroll
  for (int i = 1; i < NW; ++i) se += red[NW + i];
  const float inv = 1.f / se;
  float acc[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) acc[j] = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int r = sub + SUB * j;
    if (r < 169) {
      const int o = oc * 169 + r;
      float g = expf(yv[j] - mx) * inv;
      if (o == lab) {
        g -= 1.f;
        loss_rows[s] = mx + logf(se) - yv[j];
      }
      g *= scale;
      if (yv[j] > 0.f) conv_acc_grad(img, r / 13, r - (r / 13) * 13, av[j], g, acc);
    }
  }
  slab_write<SUB>(acc, slab + (int64_t)s * 320 + oc * 10, sub);
}

template <typename XT, int SUB, bool FUSE>
__global__ void __launch_bounds__(32 * SUB)
conv_fwd_ce_wgrad_kernel(const XT* __restrict__ x, const int64_t* __restrict__ idx,
                         const int64_t* __restrict__ labels, const float* __restrict__ w,
                         const float* __restrict__ b, float scale, float* __restrict__ slab,
                         float* __restrict__ loss_rows, const float* __restrict__ prev_slab = nullptr,
                         int Bprev = 0, float* __restrict__ pout = nullptr, SlOpt o = SlOpt{}) {
  conv_step_body<XT, SUB, FUSE>(x, idx, labels, w, b, scale, slab, loss_rows, prev_slab, Bprev, pout, o,
                                (int)blockIdx.x);
}

// One SISA local step of EVERY co-located Alice in one launch: grid (B, k), workgroup (s, a)
// runs sample s of Alice a's step with exactly conv_fwd_ce_wgrad_kernel<uint8_t, 32, true>'s
// arithmetic (bitwise the per-Alice epochs).  The per-(step, Alice) arguments come from a
// device table written once per epoch (row = this step's k descriptors; the index is
// workgroup-uniform, so they are scalar loads).  At batch 16 one Alice's step is 16
// workgroups on a 256-CU part and latency-bound; k Alices share that latency instead of
// paying it k times.
struct AliceStepDesc {
  const uint8_t* x;
  const int64_t* idx;
  const int64_t* labels;
  const float* pin;
  float* slab;
  float* loss_rows;
  const float* prev_slab;
  float* pout;
  SlOpt o;
  float scale;
  int bs, Bprev, pad;
};

__global__ void __launch_bounds__(1024)
conv_local_multi_kernel(const AliceStepDesc* __restrict__ row) {
  const AliceStepDesc& d = row[blockIdx.y];
  const int s = (int)blockIdx.x;
  if (s >= d.bs) return;                    // this Alice's last, partial batch (uniform per workgroup)
  conv_step_body<uint8_t, 32, true>(d.x, d.idx, d.labels, d.pin, nullptr, d.scale, d.slab, d.loss_rows,
                                    d.prev_slab, d.Bprev, d.pout, d.o, s);
}

// Split-mode stage 1: dW/db partials of one sample from the cut-layer gradient dy.
// 32 lanes per output channel (1024 threads), each owning pooled positions sub + 32 j
// (j < 6); all of a thread's dy / y / argmax loads are issued before the first is used,
// so the kernel is one memory round trip plus the gather-free LDS work (the 8-lane form
// with a load-then-use loop of 22 positions measured 17 us per step in --vanilla).
template <typename XT>
__global__ void __launch_bounds__(1024)
conv_wgrad_partial_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                          const uint8_t* __restrict__ am, const XT* __restrict__ x,
                          const int64_t* __restrict__ idx, float* __restrict__ slab,
                          const float* __restrict__ pslab = nullptr, int pB = 0, float* __restrict__ w = nullptr,
                          float* __restrict__ b = nullptr, float* __restrict__ s0w = nullptr,
                          float* __restrict__ s1w = nullptr, float* __restrict__ s0b = nullptr,
                          float* __restrict__ s1b = nullptr, SlOpt o = SlOpt{}) {
  __shared__ float img[IMG_LDS];
  constexpr int SUB = 32, P = (169 + SUB - 1) / SUB;
  const int s = blockIdx.x, tid = threadIdx.x;
  if (pslab && s == 0 && tid < 320) {
    // deferred mode: store the previous step's update (the values this step's forward
    // already used); nothing in this launch reads w/b or the states, and this launch's
    // own partials go to the other slab buffer
    float a0, a1;
    const float pp = conv_pending_param(w, b, s0w, s1w, s0b, s1b, pslab, pB, tid, o, a0, a1);
    const int c = tid / 10, j = tid - c * 10;
    if (j < 9) {
      if (o.kind != 0) w[c * 9 + j] = pp;
      s0w[c * 9 + j] = a0;
      if (s1w) s1w[c * 9 + j] = a1;
    } else {
      if (o.kind != 0) b[c] = pp;
      s0b[c] = a0;
      if (s1b) s1b[c] = a1;
    }
  }
  const int oc = tid / SUB, sub = tid % SUB;
  const int64_t row = (int64_t)s * 5408 + oc * 169;
  float g[P], yv[P];
  int av[P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int r = sub + SUB * j;
    const bool in = r < 169;
    g[j] = in ? dy[row + r] : 0.f;
    yv[j] = in ? y[row + r] : 0.f;
    av[j] = in ? am[row + r] : 0;
  }
  const XT* xr = x + idx[s] * 784;
  for (int i = tid; i < 784; i += 1024) img[img_idx(i / 28, i % 28)] = (float)xr[i];
  __syncthreads();
  float acc[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) acc[j] = 0.f;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int r = sub + SUB * j;
    if (r < 169 && yv[j] > 0.f) conv_acc_grad(img, r / 13, r - (r / 13) * 13, av[j], g[j], acc);
  }
  slab_write<SUB>(acc, slab + (int64_t)s * 320 + oc * 10, sub);
}

// Stage 2: g = sum over samples, optimizer update of the 288 weights + 32 biases.
__global__ void __launch_bounds__(320)
conv_opt_reduce_kernel(const float* __restrict__ slab, int B, float* __restrict__ w, float* __restrict__ b,
                       float* __restrict__ s0w, float* __restrict__ s1w, float* __restrict__ s0b,
                       float* __restrict__ s1b, SlOpt o) {
  const int p = threadIdx.x;
  float g = 0.f;
  for (int s = 0; s < B; ++s) g += slab[(int64_t)s * 320 + p];
  const int oc = p / 10, j = p - (p / 10) * 10;
  if (j < 9) {
    const int k = oc * 9 + j;
    float pp = w[k], a0 = s0w[k], a1 = s1w ? s1w[k] : 0.f;
    sl_opt_update(o, pp, g, a0, a1);
    if (o.kind != 0) w[k] = pp;
    s0w[k] = a0;
    if (s1w) s1w[k] = a1;
  } else {
    float pp = b[oc], a0 = s0b[oc], a1 = s1b ? s1b[oc] : 0.f;
    sl_opt_update(o, pp, g, a0, a1);
    if (o.kind != 0) b[oc] = pp;
    s0b[oc] = a0;
    if (s1b) s1b[oc] = a1;
  }
}

hipError_t conv_local_step(const void* x, bool x_u8, const int64_t* idx, const int64_t* labels, int B, float* w,
                           float* b, float* slab, float* loss_rows, float* s0w, float* s1w, float* s0b, float* s1b,
                           SlOpt o, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  const float scale = 1.f / (float)B;
  if (x_u8)
    conv_fwd_ce_wgrad_kernel<uint8_t, 32, false><<<B, 1024, 0, st>>>((const uint8_t*)x, idx, labels, w, b, scale, slab,
                                                                      loss_rows);
  else
    conv_fwd_ce_wgrad_kernel<float, 32, false><<<B, 1024, 0, st>>>((const float*)x, idx, labels, w, b, scale, slab,
                                                                    loss_rows);
  conv_opt_reduce_kernel<<<1, 320, 0, st>>>(slab, B, w, b, s0w, s1w, s0b, s1b, o);
  return hipGetLastError();
}

// Epoch finaliser: the last step's update from param buffer `pin` into the real tensors.
__global__ void __launch_bounds__(320)
conv_opt_finalize_kernel(const float* __restrict__ slab, int B, const float* __restrict__ pin,
                         float* __restrict__ w, float* __restrict__ b, float* __restrict__ s0w,
                         float* __restrict__ s1w, float* __restrict__ s0b, float* __restrict__ s1b, SlOpt o) {
  const int p = threadIdx.x;
  const int oc = p / 10, j = p - (p / 10) * 10;
  const int k = j < 9 ? oc * 9 + j : 288 + oc;
  float g = 0.f;
  for (int z = 0; z < B; ++z) g += slab[(int64_t)z * 320 + p];
  float pp = pin[k], a0 = pin[320 + k], a1 = pin[640 + k];
  sl_opt_update(o, pp, g, a0, a1);
  if (k < 288) {
    if (o.kind != 0) w[k] = pp;
    s0w[k] = a0;
    if (s1w) s1w[k] = a1;
  } else {
    if (o.kind != 0) b[k - 288] = pp;
    s0b[k - 288] = a0;
    if (s1b) s1b[k - 288] = a1;
  }
}

__global__ void conv_params_pack_kernel(const float* __restrict__ w, const float* __restrict__ b,
                                        const float* __restrict__ s0w, const float* __restrict__ s1w,
                                        const float* __restrict__ s0b, const float* __restrict__ s1b,
                                        float* __restrict__ P) {
  const int k = threadIdx.x;   // 320
  const bool isw = k < 288;
  P[k] = isw ? w[k] : b[k - 288];
  P[320 + k] = isw ? s0w[k] : s0b[k - 288];
  P[640 + k] = isw ? (s1w ? s1w[k] : 0.f) : (s1b ? s1b[k - 288] : 0.f);
}

// A whole SISA local epoch (ceil(n/B) steps) with the per-step optimizer folded into the
// next step's kernel: 1 launch per step + 2 for the epoch.  `ws` >= 2*B*320 + 2*960 floats.
// opt(t) gives the SlOpt of optimizer step t (host-side bias corrections).
hipError_t conv_local_epoch(const void* x, bool x_u8, const int64_t* order, int64_t n, int B, const int64_t* labels,
                            float* w, float* b, float* s0w, float* s1w, float* s0b, float* s1b, float* ws,
                            int64_t ws_elems, float* loss_rows, SlOpt (*opt)(void*, int64_t), void* optctx,
                            int64_t t0, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ws_elems < 2LL * B * 320 + 2 * 960) return hipErrorInvalidValue;
  float* slabs[2] = {ws, ws + (int64_t)B * 320};
  float* P[2] = {ws + 2LL * B * 320, ws + 2LL * B * 320 + 960};
  conv_params_pack_kernel<<<1, 320, 0, st>>>(w, b, s0w, s1w, s0b, s1b, P[0]);
  int cur = 0;
  int64_t i = 0, prevB = 0;
  for (int64_t s = 0; s < n; s += B, ++i) {
    const int bs = (int)std::min<int64_t>(B, n - s);
    const float scale = 1.f / (float)bs;
    const float* prev = i ? slabs[(i - 1) & 1] : nullptr;
    const SlOpt o = i ? opt(optctx, t0 + i - 1) : SlOpt{};
    float* pout = P[1 - cur];
    if (x_u8)
      conv_fwd_ce_wgrad_kernel<uint8_t, 32, true><<<bs, 1024, 0, st>>>((const uint8_t*)x, order + s, labels, P[cur],
                                                                       nullptr, scale, slabs[i & 1], loss_rows + s,
                                                                       prev, (int)prevB, pout, o);
    else
      conv_fwd_ce_wgrad_kernel<float, 32, true><<<bs, 1024, 0, st>>>((const float*)x, order + s, labels, P[cur],
                                                                     nullptr, scale, slabs[i & 1], loss_rows + s,
                                                                     prev, (int)prevB, pout, o);
    if (i) cur = 1 - cur;
    prevB = bs;
  }
  conv_opt_finalize_kernel<<<1, 320, 0, st>>>(slabs[(i - 1) & 1], (int)prevB, P[cur], w, b, s0w, s1w, s0b, s1b,
                                             opt(optctx, t0 + i - 1));
  return hipGetLastError();
}

// Local epochs of k co-located Alices, stepped together: step i launches ONE kernel over the
// Alices that still have a step i (Alices sorted by descending step count, so those are a
// prefix of the table row).  Each Alice keeps the single-Alice epoch's ping-pong param
// buffers and slabs (in its own `ws`) and its own optimizer step counter.
hipError_t conv_local_epoch_multi(const MultiAlice* al, int k, int B, SlOpt (*opt)(void*, int64_t), void* optctx,
                                  void* table, int64_t table_bytes, hipStream_t st) {
  if (k <= 0) return hipSuccess;
  std::vector<int> ord(k);
  int64_t nmax = 0;
  for (int a = 0; a < k; ++a) {
    ord[a] = a;
    if (al[a].ws_elems < 2LL * B * 320 + 2 * 960) return hipErrorInvalidValue;
    nmax = std::max<int64_t>(nmax, (al[a].n + B - 1) / B);
  }
  std::stable_sort(ord.begin(), ord.end(), [&](int p, int q) { return al[p].n > al[q].n; });
  if (table_bytes < (int64_t)sizeof(AliceStepDesc) * nmax * k) return hipErrorInvalidValue;
  std::vector<AliceStepDesc> host((size_t)nmax * k);
  std::vector<int> active(nmax, 0);
  std::vector<int> cur(k, 0), last_bs(k, 0);
  for (int r = 0; r < k; ++r) {
    const MultiAlice& A = al[ord[r]];
    float* slabs[2] = {A.ws, A.ws + (int64_t)B * 320};
    float* P[2] = {A.ws + 2LL * B * 320, A.ws + 2LL * B * 320 + 960};
    int c = 0;
    int64_t i = 0, prevB = 0;
    for (int64_t s = 0; s < A.n; s += B, ++i) {
      const int bs = (int)std::min<int64_t>(B, A.n - s);
      AliceStepDesc& d = host[(size_t)i * k + r];
      d.x = A.x;
      d.idx = A.order + s;
      d.labels = A.labels;
      d.pin = P[c];
      d.slab = slabs[i & 1];
      d.loss_rows = A.loss_rows + s;
      d.prev_slab = i ? slabs[(i - 1) & 1] : nullptr;
      d.pout = P[1 - c];
      d.o = i ? opt(optctx, A.t0 + i - 1) : SlOpt{};
      d.scale = 1.f / (float)bs;
      d.bs = bs;
      d.Bprev = (int)prevB;
      if (i) c = 1 - c;
      prevB = bs;
      active[i] = r + 1;
    }
    cur[ord[r]] = c;
    last_bs[ord[r]] = (int)prevB;
  }
  // the table buffer is reused from epoch to epoch: wait for the stream's earlier work (a
  // previous epoch's readers) and copy synchronously (the host table dies with this call);
  // one sync per local phase, a phase boundary anyway
  hipError_t e = hipStreamSynchronize(st);
  if (e == hipSuccess) e = hipMemcpy(table, host.data(), sizeof(AliceStepDesc) * host.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  for (int a = 0; a < k; ++a)
    conv_params_pack_kernel<<<1, 320, 0, st>>>(al[a].w, al[a].b, al[a].s0w, al[a].s1w, al[a].s0b, al[a].s1b,
                                               al[a].ws + 2LL * B * 320);
  const AliceStepDesc* tab = static_cast<const AliceStepDesc*>(table);
  for (int64_t i = 0; i < nmax; ++i)
    conv_local_multi_kernel<<<dim3(B, active[i]), 1024, 0, st>>>(tab + i * k);
  for (int a = 0; a < k; ++a) {
    const MultiAlice& A = al[a];
    if (A.n <= 0) continue;
    const int64_t ns = (A.n + B - 1) / B;
    float* slab_last = A.ws + ((ns - 1) & 1) * (int64_t)B * 320;
    float* Pc = A.ws + 2LL * B * 320 + cur[a] * 960;
    conv_opt_finalize_kernel<<<1, 320, 0, st>>>(slab_last, last_bs[a], Pc, A.w, A.b, A.s0w, A.s1w, A.s0b, A.s1b,
                                               opt(optctx, A.t0 + ns - 1));
  }
  return hipGetLastError();
}

size_t alice_step_desc_bytes() { return sizeof(AliceStepDesc); }

// Split-mode backward + optimizer.  Immediate (defer = false): partials, then the reduce +
// update launch.  Deferred (defer = true): partials only, with `pend` (the step before,
// if any) stored by workgroup 0; this step's update is left to the next forward / backward
// or to conv_apply.  Both give bitwise the same parameters.
hipError_t conv_bwd_step(const float* dy, const float* y, const uint8_t* am, const void* x, bool x_u8,
                         const int64_t* idx, int B, float* w, float* b, float* slab, float* s0w, float* s1w,
                         float* s0b, float* s1b, SlOpt o, hipStream_t st, bool defer, const ConvPending* pend) {
  if (B <= 0) return hipSuccess;
  const ConvPending p = pend ? *pend : ConvPending{nullptr, 0, nullptr, nullptr, nullptr, nullptr, SlOpt{}};
  if (x_u8)
    conv_wgrad_partial_kernel<uint8_t><<<B, 1024, 0, st>>>(dy, y, am, (const uint8_t*)x, idx, slab, p.slab, p.B, w, b,
                                                           p.s0w, p.s1w, p.s0b, p.s1b, p.o);
  else
    conv_wgrad_partial_kernel<float><<<B, 1024, 0, st>>>(dy, y, am, (const float*)x, idx, slab, p.slab, p.B, w, b,
                                                         p.s0w, p.s1w, p.s0b, p.s1b, p.o);
  if (!defer) conv_opt_reduce_kernel<<<1, 320, 0, st>>>(slab, B, w, b, s0w, s1w, s0b, s1b, o);
  return hipGetLastError();
}

// Store a deferred update (end of a deferred run, or before the weights are read).
hipError_t conv_apply(const ConvPending& p, float* w, float* b, hipStream_t st) {
  if (!p.slab || p.B <= 0) return hipSuccess;
  conv_opt_reduce_kernel<<<1, 320, 0, st>>>(p.slab, p.B, w, b, p.s0w, p.s1w, p.s0b, p.s1b, p.o);
  return hipGetLastError();
}

hipError_t conv_fwd(const void* x, bool x_u8, const int64_t* idx, int64_t row0, int B,
                    const float* w, const float* b, float* y, uint8_t* am, hipStream_t st,
                    const int64_t* lab_in, int64_t* lab_out, const ConvPending* pend) {
  if (B <= 0) return hipSuccess;
  const ConvPending p = pend ? *pend : ConvPending{nullptr, 0, nullptr, nullptr, nullptr, nullptr, SlOpt{}};
  if (x_u8)
    conv_relu_pool_fwd_kernel<uint8_t><<<dim3(B, 4), 256, 0, st>>>((const uint8_t*)x, idx, row0, w, b, y, am, lab_in,
                                                                   lab_out, p.slab, p.B, p.s0w, p.s1w, p.s0b, p.s1b,
                                                                   p.o);
  else
    conv_relu_pool_fwd_kernel<float><<<dim3(B, 4), 256, 0, st>>>((const float*)x, idx, row0, w, b, y, am, lab_in,
                                                                 lab_out, p.slab, p.B, p.s0w, p.s1w, p.s0b, p.s1b,
                                                                 p.o);
  return hipGetLastError();
}

// Frozen-front forwards of set.k Alices (uint8 shards), chunk rows per launch: one launch per
// chunk for all of them instead of one per Alice and chunk.
hipError_t conv_fwd_multi(const FrontFwdSet& set, int64_t chunk, hipStream_t st) {
  if (set.k <= 0 || set.k > kFrontFwdMax || chunk <= 0) return set.k == 0 ? hipSuccess : hipErrorInvalidValue;
  int64_t nmax = 0;
  for (int a = 0; a < set.k; ++a) nmax = std::max<int64_t>(nmax, set.d[a].n);
  for (int64_t r0 = 0; r0 < nmax; r0 += chunk) {
    const int rows = (int)std::min<int64_t>(chunk, nmax - r0);
    conv_fwd_multi_kernel<<<dim3(rows, 4, set.k), 256, 0, st>>>(set, r0);
  }
  return hipGetLastError();
}

}  // namespace sl
