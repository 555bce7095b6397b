// Fused softmax-cross-entropy forward+backward and fused evaluation counters.
//
// Reference ops: nn.CrossEntropyLoss (mean) on Bob's 100 logits
// (data_entities_vanilla.py:229-230, data_entities_vanilla_sisa.py:307-308), on the
// U-shape head's 10 logits (data_entities.py:76) and on the SISA Alice's 5408-wide
// activation treated as logits (Q5, data_entities_vanilla_sisa.py:64-65); and the
// torch.max + mask counting of eval_breakdown (data_entities_vanilla.py:181-194).
// SURVEY §2.7 K9, K10.  One wave64 per row; all reductions are in-register
// shuffles, no LDS.
#include "common.h"

namespace sl {

// loss_rows[m] = logsumexp(x_m) - x_m[y_m];  d[m,:] = scale * (softmax(x_m) - onehot(y_m)).
// Rows with label == ignore get loss 0 and a zero gradient row.
__global__ void __launch_bounds__(256)
softmax_ce_kernel(const float* __restrict__ x, int ldx, const int64_t* __restrict__ y, int64_t ignore,
                  float scale, float* __restrict__ loss_rows, float* __restrict__ d, int ldd, int M, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (int64_t)row * ldx;
  float* dr = d ? d + (int64_t)row * ldd : nullptr;
  const int64_t lab = y[row];
  if (lab == ignore) {
    if (lane == 0) loss_rows[row] = 0.f;
    if (dr)
      for (int c = lane; c < C; c += 64) dr[c] = 0.f;
    return;
  }
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, xr[c]);
  mx = sl_wave_max(mx);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += expf(xr[c] - mx);
  s = sl_wave_sum(s);
  const float inv = 1.f / s;
  const float lse = mx + logf(s);
  if (lane == 0) loss_rows[row] = lse - xr[lab];
  if (dr) {
    for (int c = lane; c < C; c += 64) {
      float p = expf(xr[c] - mx) * inv;
      if (c == lab) p -= 1.f;
      dr[c] = p * scale;
    }
  }
}

// Wide rows (C in the thousands, e.g. the 5408-way SISA client loss): one 256-thread
// workgroup per row, LDS reduction across its 4 waves.
__global__ void __launch_bounds__(256)
softmax_ce_wide_kernel(const float* __restrict__ x, int ldx, const int64_t* __restrict__ y, int64_t ignore,
                       float scale, float* __restrict__ loss_rows, float* __restrict__ d, int ldd, int C) {
  __shared__ float red[8];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* xr = x + (int64_t)row * ldx;
  float* dr = d ? d + (int64_t)row * ldd : nullptr;
  const int64_t lab = y[row];
  if (lab == ignore) {
    if (tid == 0) loss_rows[row] = 0.f;
    if (dr)
      for (int c = tid; c < C; c += 256) dr[c] = 0.f;
    return;
  }
  float mx = -INFINITY;
  for (int c = tid; c < C; c += 256) mx = fmaxf(mx, xr[c]);
  mx = sl_wave_max(mx);
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
  for (int c = tid; c < C; c += 256) s += expf(xr[c] - mx);
  s = sl_wave_sum(s);
  if (lane == 0) red[4 + wv] = s;
  __syncthreads();
  s = red[4] + red[5] + red[6] + red[7];
  const float inv = 1.f / s;
  if (tid == 0) loss_rows[row] = mx + logf(s) - xr[lab];
  if (dr) {
    for (int c = tid; c < C; c += 256) {
      float p = expf(xr[c] - mx) * inv;
      if (c == lab) p -= 1.f;
      dr[c] = p * scale;
    }
  }
}

// counters[6] += {correct, total, correct_unlearned, total_unlearned, correct_remaining, total_remaining}
__global__ void __launch_bounds__(256)
eval_counters_kernel(const float* __restrict__ x, int ldx, const int64_t* __restrict__ y, int64_t omit,
                     unsigned long long* __restrict__ counters, int M, int C) {
  __shared__ unsigned int part[6];
  if (threadIdx.x < 6) part[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row < M) {
    const float* xr = x + (int64_t)row * ldx;
    float best = -INFINITY;
    int arg = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float v = xr[c];
      if (v > best) { best = v; arg = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oa = __shfl_xor(arg, o, 64);
      if (ob > best || (ob == best && oa < arg)) { best = ob; arg = oa; }
    }
    if (lane == 0) {
      const int64_t lab = y[row];
      const unsigned ok = (arg == lab) ? 1u : 0u;
      atomicAdd(&part[0], ok);
      atomicAdd(&part[1], 1u);
      if (lab == omit) { atomicAdd(&part[2], ok); atomicAdd(&part[3], 1u); }
      else { atomicAdd(&part[4], ok); atomicAdd(&part[5], 1u); }
    }
  }
  __syncthreads();
  if (threadIdx.x < 6 && part[threadIdx.x]) atomicAdd(&counters[threadIdx.x], (unsigned long long)part[threadIdx.x]);
}

// ReLU / dropout backward of a layer's own output: out = dout * scale * [h > 0] (the last
// layer of the U-shape middle, model2's fc2 + ReLU).  One launch instead of three eager
// elementwise ops (compare, multiply, multiply).
__global__ void __launch_bounds__(256)
relu_mask_kernel(const float* __restrict__ d, const float* __restrict__ h, float scale, float* __restrict__ out,
                 int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = h[i] > 0.f ? d[i] * scale : 0.f;
}

hipError_t relu_mask(const float* d, const float* h, float scale, float* out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  relu_mask_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d, h, scale, out, n);
  return hipGetLastError();
}

hipError_t softmax_ce(const float* x, int ldx, const int64_t* y, int64_t ignore, float scale, float* loss_rows,
                      float* d, int ldd, int M, int C, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (C > 512)
    softmax_ce_wide_kernel<<<M, 256, 0, st>>>(x, ldx, y, ignore, scale, loss_rows, d, ldd, C);
  else
    softmax_ce_kernel<<<(M + 3) / 4, 256, 0, st>>>(x, ldx, y, ignore, scale, loss_rows, d, ldd, M, C);
  return hipGetLastError();
}

hipError_t eval_counters(const float* x, int ldx, const int64_t* y, int64_t omit, unsigned long long* counters,
                         int M, int C, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  eval_counters_kernel<<<(M + 3) / 4, 256, 0, st>>>(x, ldx, y, omit, counters, M, C);
  return hipGetLastError();
}


// U-shape head (reference model3 = Linear(100, 10) + CrossEntropyLoss on Alice,
// data_entities.py:74-81): forward, softmax-CE, data gradient and the optimizer step of
// the whole layer in ONE workgroup (the separate path is four launches of a few us each
// for 1,010 parameters).  dX uses the weights before the update; with mask_dx it is also
// masked by [X > 0], the ReLU backward of the layer that produced X (Bob's model2 ends in a
// ReLU whose output X is), so the producer skips its own mask launch.  M*K, C*K <= 4096.
__global__ void __launch_bounds__(256)
head_step_kernel(const float* __restrict__ X, const float* __restrict__ W, const float* __restrict__ bias,
                 const int64_t* __restrict__ y, int64_t ignore, float scale, float* __restrict__ loss_rows,
                 float* __restrict__ dX, float* __restrict__ Wout, float* __restrict__ bout, float* __restrict__ s0w,
                 float* __restrict__ s1w, float* __restrict__ s0b, float* __restrict__ s1b, int M, int K, int C,
                 SlOpt o, int mask_dx, int bf) {
  // bf: bf16 compute (`--dtype bf16`): every product's operands rounded to bf16, fp32 sums;
  // the master weights the optimizer updates stay fp32
  auto R = [bf](float v) { return bf ? bfr(v) : v; };
  __shared__ float sx[4096];
  __shared__ float sw[4096];
  __shared__ float sd[1024];     // dlogits [M][C]
  const int tid = threadIdx.x;
  // the optimizer state this thread updates at the end is loaded first, so the update does
  // not wait on dependent global loads (4 elements per thread covers C*K <= 1024)
  constexpr int PF = 4;
  float r0[PF], r1[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int i = tid + 256 * j;
    r0[j] = i < C * K ? s0w[i] : 0.f;
    r1[j] = (i < C * K && s1w) ? s1w[i] : 0.f;
  }
  float rb0 = 0.f, rb1 = 0.f, rbp = 0.f;
  if (bias && tid < C) {
    rbp = bias[tid];
    rb0 = s0b[tid];
    rb1 = s1b ? s1b[tid] : 0.f;
  }
  for (int i = tid; i < M * K; i += 256) sx[i] = X[i];
  for (int i = tid; i < C * K; i += 256) sw[i] = W[i];
  __syncthreads();
  // logits (into sd), one (m, c) per thread
  for (int i = tid; i < M * C; i += 256) {
    const int m = i / C, c = i - m * C;
    float v = 0.f;
    for (int k = 0; k < K; ++k) v = fmaf(R(sx[m * K + k]), R(sw[c * K + k]), v);
    sd[i] = v + (bias ? bias[c] : 0.f);
  }
  __syncthreads();
  // softmax-CE per row
  if (tid < M) {
    float* r = sd + tid * C;
    const int64_t lab = y[tid];
    if (lab == ignore) {
      loss_rows[tid] = 0.f;
      for (int c = 0; c < C; ++c) r[c] = 0.f;
    } else {
      float mx = -INFINITY;
      for (int c = 0; c < C; ++c) mx = fmaxf(mx, r[c]);
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(r[c] - mx);
      const float inv = 1.f / se;
      loss_rows[tid] = mx + logf(se) - r[lab];
      for (int c = 0; c < C; ++c) {
        float p = expf(r[c] - mx) * inv;
        if (c == lab) p -= 1.f;
        r[c] = p * scale;
      }
    }
  }
  __syncthreads();
  // data gradient with the current weights
  for (int i = tid; i < M * K; i += 256) {
    const int m = i / K, k = i - m * K;
    float v = 0.f;
    for (int c = 0; c < C; ++c) v = fmaf(R(sd[m * C + c]), R(sw[c * K + k]), v);
    dX[i] = (mask_dx && !(sx[i] > 0.f)) ? 0.f : v;   // mask_dx: the producer's ReLU backward too
  }
  // weight / bias gradient and the optimizer step
  auto wstep = [&](int i, float a0, float a1) {
    const int c = i / K, k = i - c * K;
    float g = 0.f;
    for (int m = 0; m < M; ++m) g = fmaf(R(sd[m * C + c]), R(sx[m * K + k]), g);
    float pp = sw[i];
    sl_opt_update(o, pp, g, a0, a1);
    if (o.kind != 0) Wout[i] = pp;
    s0w[i] = a0;
    if (s1w) s1w[i] = a1;
  };
#pragma unroll
  for (int j = 0; j < PF; ++j)       // compile-time register index (no scratch)
    if (tid + 256 * j < C * K) wstep(tid + 256 * j, r0[j], r1[j]);
  for (int i = tid + 256 * PF; i < C * K; i += 256) wstep(i, s0w[i], s1w ? s1w[i] : 0.f);
  if (bias && tid < C) {
    float g = 0.f;
    for (int m = 0; m < M; ++m) g += sd[m * C + tid];
    float pp = rbp, a0 = rb0, a1 = rb1;
    sl_opt_update(o, pp, g, a0, a1);
    if (o.kind != 0) bout[tid] = pp;
    s0b[tid] = a0;
    if (s1b) s1b[tid] = a1;
  }
}

// head_step_mfma_kernel: the same step for M <= 16 rows, C <= 16 classes, K <= 128 (% 4)
// features — the U-shape head (16 x 100 -> 10) — with its three products on exact-fp32 MFMA
// (v_mfma_f32_16x16x4f32, 16 x 16 tiles) instead of per-thread FMA chains: logits (wave 0,
// K / 4 steps), data gradient (one 16-column tile of K per wave step, C padded to 16) and
// weight gradient (M = 16 as the reduction), the softmax-CE on DPP row reductions over the
// 16 class lanes of each row.  bf16 compute is a template parameter.  One 256-thread
// workgroup; the optimizer update keeps head_step_kernel's thread mapping (state loads first).
template <bool BF>
__global__ void __launch_bounds__(256)
head_step_mfma_kernel(const float* __restrict__ X, const float* __restrict__ W, const float* __restrict__ bias,
                      const int64_t* __restrict__ y, int64_t ignore, float scale, float* __restrict__ loss_rows,
                      float* __restrict__ dX, float* __restrict__ Wout, float* __restrict__ bout,
                      float* __restrict__ s0w, float* __restrict__ s1w, float* __restrict__ s0b,
                      float* __restrict__ s1b, int M, int K, int C, SlOpt o, int mask_dx) {
  constexpr int KP = 132;                      // padded LDS row (K <= 128)
  __shared__ __attribute__((aligned(16))) float sx[16][KP];
  __shared__ __attribute__((aligned(16))) float sw[16][KP];
  __shared__ __attribute__((aligned(16))) float sg[16][KP];    // dW [C][K]
  __shared__ float sd[16][17];                 // dlogits [M][C]
  auto R = [](float v) { return BF ? bfr(v) : v; };
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lq = lane >> 4;
  constexpr int PF = 8;                        // state elements per thread (C K <= 2048)
  float r0[PF], r1[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int i = tid + 256 * j;
    r0[j] = i < C * K ? s0w[i] : 0.f;
    r1[j] = (i < C * K && s1w) ? s1w[i] : 0.f;
  }
  float rb0 = 0.f, rb1 = 0.f, rbp = 0.f;
  if (bias && tid < C) {
    rbp = bias[tid];
    rb0 = s0b[tid];
    rb1 = s1b ? s1b[tid] : 0.f;
  }
  // operands into LDS, zero-padded to 16 rows and 16-column tiles: every float4 load of X and
  // W is issued before anything is stored (one memory round trip), the zero fill meanwhile
  const int K4 = K >> 2;
  f32x4 xr[2], wr[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int f = tid + 256 * j, r = f / K4, q = f - r * K4;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    xr[j] = r < M ? reinterpret_cast<const f32x4*>(X)[f] : z4;
    wr[j] = r < C ? reinterpret_cast<const f32x4*>(W)[f] : z4;
  }
  for (int i = tid; i < 16 * KP; i += 256) {
    (&sx[0][0])[i] = 0.f;
    (&sw[0][0])[i] = 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int f = tid + 256 * j, r = f / K4, q = f - r * K4;
    if (r < 16) {
      *reinterpret_cast<f32x4*>(&sx[r][4 * q]) = xr[j];
      *reinterpret_cast<f32x4*>(&sw[r][4 * q]) = wr[j];
    }
  }
  __syncthreads();
  // logits D[m][c] = sum_k X[m][k] W[c][k] (wave 0): A lane (m = li, k = 4s + lq), B (k, c = li)
  if (wv == 0) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s4 = 0; s4 < K; s4 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(R(sx[li][s4 + lq]), R(sw[li][s4 + lq]), acc, 0, 0, 0);
    // lane (c = li, lq) holds rows m = 4 lq + r; softmax over the 16 class lanes of each row
    const bool vc = li < C;
    const float bc = (bias && vc) ? bias[li] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * lq + r;
      const float z = vc ? acc[r] + bc : -INFINITY;
      const float mx = sl_row16_max(z);
      const float e = vc ? expf(z - mx) : 0.f;
      const float se = sl_row16_sum(e);
      float dl = 0.f;
      if (m < M) {
        const int64_t lab = y[m];
        if (lab == ignore) {
          if (li == 0) loss_rows[m] = 0.f;
        } else {
          const float zl = sl_dpp_pick(z, (int)lab);
          if (li == 0) loss_rows[m] = mx + logf(se) - zl;
          if (vc) dl = (e / se - (li == lab ? 1.f : 0.f)) * scale;
        }
      }
      sd[m][li] = dl;
    }
  }
  __syncthreads();
  // data gradient dX[m][k] = sum_c dlog[m][c] W[c][k]: wave w takes 16-column tiles w, w+4, ..
  for (int kt = wv; kt * 16 < K; kt += 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(R(sd[li][s4 + lq]), R(sw[s4 + lq][16 * kt + li]), acc, 0, 0, 0);
    const int k = 16 * kt + li;
    if (k < K) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * lq + r;
        if (m < M) dX[m * K + k] = (mask_dx && !(sx[m][k] > 0.f)) ? 0.f : acc[r];
      }
    }
  }
  // weight gradient dW[c][k] = sum_m dlog[m][c] X[m][k] -> LDS
  for (int kt = wv; kt * 16 < K; kt += 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(R(sd[s4 + lq][li]), R(sx[s4 + lq][16 * kt + li]), acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) sg[4 * lq + r][16 * kt + li] = acc[r];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int i = tid + 256 * j;
    if (i < C * K) {
      const int c = i / K, k = i - c * K;
      float pp = sw[c][k], a0 = r0[j], a1 = r1[j];
      sl_opt_update(o, pp, sg[c][k], a0, a1);
      if (o.kind != 0) Wout[i] = pp;
      s0w[i] = a0;
      if (s1w) s1w[i] = a1;
    }
  }
  if (bias && tid < C) {
    float g = 0.f;
    for (int m = 0; m < M; ++m) g += sd[m][tid];
    float pp = rbp, a0 = rb0, a1 = rb1;
    sl_opt_update(o, pp, g, a0, a1);
    if (o.kind != 0) bout[tid] = pp;
    s0b[tid] = a0;
    if (s1b) s1b[tid] = a1;
  }
}

hipError_t head_step(const float* X, float* W, float* b, const int64_t* y, int64_t ignore, float scale,
                     float* loss_rows, float* dX, float* s0w, float* s1w, float* s0b, float* s1b, int M, int K, int C,
                     SlOpt o, bool mask_dx, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (M * K > 4096 || C * K > 4096 || M * C > 1024) return hipErrorInvalidValue;
  const bool al = ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) == 0;
  if (M <= 16 && C <= 16 && K <= 128 && (K & 3) == 0 && C * K <= 2048 && al) {
    if (g_bf16)
      head_step_mfma_kernel<true><<<1, 256, 0, st>>>(X, W, b, y, ignore, scale, loss_rows, dX, W, b, s0w, s1w, s0b,
                                                     s1b, M, K, C, o, mask_dx ? 1 : 0);
    else
      head_step_mfma_kernel<false><<<1, 256, 0, st>>>(X, W, b, y, ignore, scale, loss_rows, dX, W, b, s0w, s1w, s0b,
                                                      s1b, M, K, C, o, mask_dx ? 1 : 0);
    return hipGetLastError();
  }
  head_step_kernel<<<1, 256, 0, st>>>(X, W, b, y, ignore, scale, loss_rows, dX, W, b, s0w, s1w, s0b, s1b, M, K, C, o,
                                      mask_dx ? 1 : 0, g_bf16);
  return hipGetLastError();
}

}  // namespace sl
