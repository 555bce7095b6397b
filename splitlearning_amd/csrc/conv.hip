// Client-front kernels: fused gather + conv3x3(1->32) + bias + ReLU + maxpool2x2
// forward, and fused pool/ReLU backward + weight/bias gradient + optimizer step.
//
// Reference ops: models.py:8-9,21-23 (Conv2d(1,32,3) -> ReLU -> MaxPool(2,2)),
// trained with Adam(wd=1e-5) (data_entities_vanilla_sisa.py:48) or SGD-m via the
// DistributedOptimizer (data_entities_vanilla.py:37-42).  SURVEY §2.7 K1-K3, K13.
//
// The conv has K = 9 (one input channel), far too small for MFMA, so it is a
// direct LDS-tiled convolution: one 256-thread workgroup per sample stages the
// 28x28 image (converted from the uint8 shard row it gathers itself, so there
// is no separate collate/convert kernel) and 32x9 weights in LDS and writes the
// pooled, NCHW-flattened [5408] activation plus a 2-bit argmax for backward.
#include "common.h"

namespace sl {

template <typename XT>
__global__ void __launch_bounds__(256)
conv_relu_pool_fwd_kernel(const XT* __restrict__ x, const int64_t* __restrict__ idx, int64_t row0,
                          const float* __restrict__ w, const float* __restrict__ b,
                          float* __restrict__ y, uint8_t* __restrict__ am) {
  __shared__ float img[28 * 28];
  __shared__ float sw[32 * 9];
  __shared__ float sb[32];
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t src = idx ? idx[s] : row0 + s;
  const XT* xr = x + src * 784;
  for (int i = tid; i < 784; i += 256) img[i] = (float)xr[i];
  for (int i = tid; i < 288; i += 256) sw[i] = w[i];
  if (tid < 32) sb[tid] = b[tid];
  __syncthreads();
  float* yo = y + (int64_t)s * 5408;
  uint8_t* ao = am + (int64_t)s * 5408;
  for (int o = tid; o < 5408; o += 256) {
    const int oc = o / 169;
    const int r = o - oc * 169;
    const int ph = r / 13;
    const int pw = r - ph * 13;
    const float* wk = sw + oc * 9;
    const float* base = img + (2 * ph) * 28 + 2 * pw;
    float patch[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) patch[i][j] = base[i * 28 + j];
    float best = 0.f;
    int arg = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float acc = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) acc = fmaf(wk[kh * 3 + kw], patch[dy + kh][dx + kw], acc);
        acc += sb[oc];
        const int pos = dy * 2 + dx;
        if (pos == 0 || acc > best) { best = acc; arg = pos; }   // first max (torch order)
      }
    yo[o] = fmaxf(best, 0.f);
    ao[o] = (uint8_t)arg;
  }
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

__device__ __forceinline__ void conv_pool_at(const float* img, const float* wk, float bias, int ph, int pw,
                                             float& y, int& arg) {
  const float* base = img + (2 * ph) * 28 + 2 * pw;
  float patch[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) patch[i][j] = base[i * 28 + j];
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

__device__ __forceinline__ void conv_acc_grad(const float* img, int ph, int pw, int a, float g, float* acc) {
  const float* xr = img + (2 * ph + (a >> 1)) * 28 + 2 * pw + (a & 1);
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] = fmaf(g, xr[kh * 28 + kw], acc[kh * 3 + kw]);
  acc[9] += g;
}

__device__ __forceinline__ void slab_write8(float* acc, float* dst, int sub) {
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    float v = acc[j];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    acc[j] = v;
  }
  if (sub == 0) {
#pragma unroll
    for (int j = 0; j < 10; ++j) dst[j] = acc[j];
  }
}

template <typename XT>
__device__ __forceinline__ void stage_sample(const XT* x, int64_t src, const float* w, const float* b, float* img,
                                             float* sw, float* sb) {
  const int tid = threadIdx.x;
  const XT* xr = x + src * 784;
  for (int i = tid; i < 784; i += 256) img[i] = (float)xr[i];
  for (int i = tid; i < 288; i += 256) sw[i] = w[i];
  if (tid < 32) sb[tid] = b[tid];
  __syncthreads();
}

// SISA local step, stage 1: forward + softmax-CE over the 5408-wide activation + dW/db partials.
template <typename XT>
__global__ void __launch_bounds__(256)
conv_fwd_ce_wgrad_kernel(const XT* __restrict__ x, const int64_t* __restrict__ idx,
                         const int64_t* __restrict__ labels, const float* __restrict__ w,
                         const float* __restrict__ b, float scale, float* __restrict__ slab,
                         float* __restrict__ loss_rows) {
  __shared__ float img[28 * 28];
  __shared__ float sw[32 * 9];
  __shared__ float sb[32];
  __shared__ float red[8];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int64_t src = idx[s];
  stage_sample(x, src, w, b, img, sw, sb);
  const int oc = tid >> 3, sub = tid & 7;
  const float* wk = sw + oc * 9;
  const float bias = sb[oc];
  float yv[22];
  int av[22];
  float mx = 0.f;   // activations are >= 0 after ReLU
#pragma unroll
  for (int j = 0; j < 22; ++j) {
    const int r = sub + 8 * j;
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
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < 22; ++j)
    if (sub + 8 * j < 169) se += expf(yv[j] - mx);
  se = sl_wave_sum(se);
  if (lane == 0) red[4 + wv] = se;
  __syncthreads();
  se = red[4] + red[5] + red[6] + red[7];
  const float inv = 1.f / se;
  const int64_t lab = labels[src];
  float acc[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) acc[j] = 0.f;
#pragma unroll
  for (int j = 0; j < 22; ++j) {
    const int r = sub + 8 * j;
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
  slab_write8(acc, slab + (int64_t)s * 320 + oc * 10, sub);
}

// Split-mode stage 1: dW/db partials of one sample from the cut-layer gradient dy.
template <typename XT>
__global__ void __launch_bounds__(256)
conv_wgrad_partial_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                          const uint8_t* __restrict__ am, const XT* __restrict__ x,
                          const int64_t* __restrict__ idx, float* __restrict__ slab) {
  __shared__ float img[28 * 28];
  const int s = blockIdx.x, tid = threadIdx.x;
  const XT* xr = x + idx[s] * 784;
  for (int i = tid; i < 784; i += 256) img[i] = (float)xr[i];
  __syncthreads();
  const int oc = tid >> 3, sub = tid & 7;
  float acc[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) acc[j] = 0.f;
  const int64_t row = (int64_t)s * 5408 + oc * 169;
  for (int r = sub; r < 169; r += 8) {
    if (y[row + r] > 0.f) conv_acc_grad(img, r / 13, r - (r / 13) * 13, am[row + r], dy[row + r], acc);
  }
  slab_write8(acc, slab + (int64_t)s * 320 + oc * 10, sub);
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
    conv_fwd_ce_wgrad_kernel<uint8_t><<<B, 256, 0, st>>>((const uint8_t*)x, idx, labels, w, b, scale, slab, loss_rows);
  else
    conv_fwd_ce_wgrad_kernel<float><<<B, 256, 0, st>>>((const float*)x, idx, labels, w, b, scale, slab, loss_rows);
  conv_opt_reduce_kernel<<<1, 320, 0, st>>>(slab, B, w, b, s0w, s1w, s0b, s1b, o);
  return hipGetLastError();
}

hipError_t conv_bwd_step(const float* dy, const float* y, const uint8_t* am, const void* x, bool x_u8,
                         const int64_t* idx, int B, float* w, float* b, float* slab, float* s0w, float* s1w,
                         float* s0b, float* s1b, SlOpt o, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (x_u8)
    conv_wgrad_partial_kernel<uint8_t><<<B, 256, 0, st>>>(dy, y, am, (const uint8_t*)x, idx, slab);
  else
    conv_wgrad_partial_kernel<float><<<B, 256, 0, st>>>(dy, y, am, (const float*)x, idx, slab);
  conv_opt_reduce_kernel<<<1, 320, 0, st>>>(slab, B, w, b, s0w, s1w, s0b, s1b, o);
  return hipGetLastError();
}

hipError_t conv_fwd(const void* x, bool x_u8, const int64_t* idx, int64_t row0, int B,
                    const float* w, const float* b, float* y, uint8_t* am, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (x_u8)
    conv_relu_pool_fwd_kernel<uint8_t><<<B, 256, 0, st>>>((const uint8_t*)x, idx, row0, w, b, y, am);
  else
    conv_relu_pool_fwd_kernel<float><<<B, 256, 0, st>>>((const float*)x, idx, row0, w, b, y, am);
  return hipGetLastError();
}

}  // namespace sl
