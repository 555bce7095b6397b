// Server-step fusions for Bob's 3-layer tail (fc1 ReLU+Dropout, fc2 ReLU+Dropout, fc3 ->
// cross-entropy; reference model2_sisa, models.py:46-63, trained per batch with Adam or SGD-m).
//
// At B = 16 the step is HBM-bound in fc1/fc2 and launch-bound everywhere else: the eager
// chain is 13 kernels, each with a ~1.5-2.5 us dependent-launch boundary, and on a
// tensor-parallel shard (1/8 of the bytes) the boundaries dominate.  Two fusions:
//
//  head3_kernel  one workgroup per batch row: reduce fc2's split-K partial slabs, apply
//                fc2's bias/ReLU/dropout (-> h2), fc3 logits, softmax-CE (loss, dlogits),
//                fc3 data gradient and fc2's ReLU/dropout backward (-> dz2).  Replaces
//                fc2-epilogue, fc3-forward(+epilogue), CE and fc3-dgrad (5 launches).
//                fc3 is 100x1000: each workgroup streams W3 twice from L2.
//
//  wgrad_group_kernel   the fused wgrad+optimizer (v3 layout) for up to 3 layers in one
//                launch; a layer's dZ may be given as un-reduced split-N partial slabs plus
//                a ReLU/dropout mask, reduced while staging into LDS (replaces the dgrad
//                reduce kernel).
#include "fused.h"

namespace sl {

__global__ void __launch_bounds__(256)
head3_kernel(const float* __restrict__ P2, int S2, int64_t slab2, Epi e2, const float* __restrict__ W3,
             const float* __restrict__ b3, const int64_t* __restrict__ y, int64_t ignore, float scale,
             float* __restrict__ h2, float* __restrict__ dlog, float* __restrict__ dz2,
             float* __restrict__ loss_rows, int N2, int C) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* hrow = sm;            // N2 (rounded up to 4)
  float* lg = sm + ((N2 + 3) & ~3);   // C
  // grid (M, Q): workgroup (m, q) recomputes row m's logits and CE (cheap, L2-resident W3)
  // but owns only column quarter q of the h2 / dz2 outputs, so the dz2 phase is spread
  // over M*Q workgroups.
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int Q = gridDim.y, q = blockIdx.y;
  const int n4 = N2 >> 2;   // N2 % 4 == 0 (checked on the host)
  const int q4a = (int)(((int64_t)n4 * q) / Q), q4b = (int)(((int64_t)n4 * (q + 1)) / Q);
  // 1. h2 = epilogue(sum of fc2 partial slabs); float4 per thread, slab loads unrolled so
  //    they are all in flight together
  const float* prow = P2 + (int64_t)m * N2;
  for (int c4 = tid; c4 < n4; c4 += 256) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int s = 0; s < S2; ++s) v += reinterpret_cast<const f32x4*>(prow + s * slab2)[c4];
    f32x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = apply_epi(e2, v[i], m, 4 * c4 + i);
    reinterpret_cast<f32x4*>(hrow)[c4] = o;
    if (c4 >= q4a && c4 < q4b) reinterpret_cast<f32x4*>(h2 + (int64_t)m * N2)[c4] = o;
  }
  __syncthreads();
  // 2. logits[o] = <h2, W3[o]> + b3[o]: a wave takes OG outputs at a time (OG independent
  //    accumulators / loads in flight), lanes split K in float4 steps
  constexpr int OG = 5;
  const f32x4* hr = reinterpret_cast<const f32x4*>(hrow);
  for (int o0 = wv * OG; o0 < C; o0 += 4 * OG) {
    float acc[OG];
#pragma unroll
    for (int j = 0; j < OG; ++j) acc[j] = 0.f;
#pragma unroll 4
    for (int qq = lane; qq < n4; qq += 64) {
      const f32x4 a = hr[qq];
#pragma unroll
      for (int j = 0; j < OG; ++j) {
        if (o0 + j < C) {
          const f32x4 b = reinterpret_cast<const f32x4*>(W3 + (int64_t)(o0 + j) * N2)[qq];
          acc[j] = fmaf(a[0], b[0], fmaf(a[1], b[1], fmaf(a[2], b[2], fmaf(a[3], b[3], acc[j]))));
        }
      }
    }
#pragma unroll
    for (int j = 0; j < OG; ++j) {
      const float s = sl_wave_sum(acc[j]);
      if (lane == 0 && o0 + j < C) lg[o0 + j] = s + (b3 ? b3[o0 + j] : 0.f);
    }
  }
  __syncthreads();
  // 3. softmax cross-entropy of the row (wave 0)
  const int64_t lab = y[m];
  if (wv == 0) {
    if (lab == ignore) {
      for (int c = lane; c < C; c += 64) lg[c] = 0.f;
      if (lane == 0 && q == 0) loss_rows[m] = 0.f;
    } else {
      float mx = -INFINITY;
      for (int c = lane; c < C; c += 64) mx = fmaxf(mx, lg[c]);
      mx = sl_wave_max(mx);
      float se = 0.f;
      for (int c = lane; c < C; c += 64) se += expf(lg[c] - mx);
      se = sl_wave_sum(se);
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
    for (int c = tid; c < C; c += 256) dlog[(int64_t)m * C + c] = lg[c];
  // 4. dz2 = (dlogits . W3) * dscale * [h2 > 0] for this workgroup's column slice: the
  //    slice's float4 columns x the C outputs are spread over all 256 threads (OGR output
  //    groups per column), partial sums reduced through LDS (reuses the logits' tail).
  const int ncol = q4b - q4a;                 // float4 columns of this slice (<= 64)
  const int ogr = ncol > 0 ? max(1, 256 / ncol) : 1;
  __shared__ f32x4 part[256];
  {
    const int col = tid % max(ncol, 1), grp = tid / max(ncol, 1);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (ncol > 0 && grp < ogr) {
      const int qq = q4a + col;
#pragma unroll 4
      for (int o = grp; o < C; o += ogr) acc += lg[o] * reinterpret_cast<const f32x4*>(W3 + (int64_t)o * N2)[qq];
    }
    part[tid] = acc;
  }
  __syncthreads();
  if (tid < ncol) {
    f32x4 acc = part[tid];
    for (int gI = 1; gI < ogr; ++gI) acc += part[gI * ncol + tid];
    const int qq = q4a + tid;
    const f32x4 h = reinterpret_cast<const f32x4*>(hrow)[qq];
    f32x4 out;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = h[i] > 0.f ? acc[i] * e2.dscale : 0.f;
    reinterpret_cast<f32x4*>(dz2 + (int64_t)m * N2)[qq] = out;
  }
}

template <bool ADAM>
__global__ void __launch_bounds__(1024)
wgrad_group_kernel(WgGroup grp, int M, SlOpt o) {
  __shared__ f32x4 sa[16][64];
  __shared__ float sdz[16][16];
  // pick the layer with selects (no runtime-indexed access to the by-value argument)
  const int by = (int)blockIdx.y;
  const WgDesc L = (grp.n > 2 && by >= grp.d[2].yb0) ? grp.d[2]
                   : ((grp.n > 1 && by >= grp.d[1].yb0) ? grp.d[1] : grp.d[0]);
  const int kb = blockIdx.x * 256;
  if (kb >= L.K) return;                 // uniform per workgroup
  const int tid = threadIdx.x;
  const int r = tid >> 6, lane = tid & 63;
  const int n0 = ((int)blockIdx.y - L.yb0) * 16;
  const int n = n0 + r;
  const int k = kb + lane * 4;
  const bool act = (n < L.N) && (k < L.K);
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  const int64_t off = (int64_t)n * L.ldw + k;
  f32x4 p = zv, q0 = zv, q1 = zv;
  if (act) {
    p = *reinterpret_cast<const f32x4*>(L.W + off);
    q0 = *reinterpret_cast<const f32x4*>(L.s0 + off);
    if (ADAM) q1 = *reinterpret_cast<const f32x4*>(L.s1 + off);
  }
  f32x4 g = zv;
  float gb = 0.f;
  for (int mc = 0; mc < M; mc += 16) {
    if (mc) __syncthreads();
    {
      const int mm = mc + r;
      sa[r][lane] = (mm < M && k < L.K) ? *reinterpret_cast<const f32x4*>(L.A + (int64_t)mm * L.lda + k) : zv;
      if (tid < 256) {
        const int mr = mc + (tid >> 4), nn = n0 + (tid & 15);
        float v = 0.f;
        if (mr < M && nn < L.N) {
          if (L.dzp) {
            for (int s = 0; s < L.S; ++s) v += L.dzp[s * L.slab + (int64_t)mr * L.N + nn];
            if (L.hmask) v = L.hmask[(int64_t)mr * L.N + nn] > 0.f ? v * L.mscale : 0.f;
          } else {
            v = L.dz[(int64_t)mr * L.ldz + nn];
          }
        }
        sdz[tid >> 4][tid & 15] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int mm = 0; mm < 16; ++mm) {
      const float d = sdz[mm][r];
      g += d * sa[mm][lane];
      gb += d;
    }
  }
  if (act) {
    sl_opt_update4<ADAM>(o, p, g, q0, q1);
    if (o.kind != 0) *reinterpret_cast<f32x4*>(L.W + off) = p;
    *reinterpret_cast<f32x4*>(L.s0 + off) = q0;
    if (ADAM) *reinterpret_cast<f32x4*>(L.s1 + off) = q1;
  }
  if (L.bias && blockIdx.x == 0 && lane == 0 && n < L.N) {
    float pb = L.bias[n], b0 = L.sb0[n], b1 = L.sb1 ? L.sb1[n] : 0.f;
    sl_opt_update(o, pb, gb, b0, b1);
    if (o.kind != 0) L.bias[n] = pb;
    L.sb0[n] = b0;
    if (L.sb1) L.sb1[n] = b1;
  }
}

hipError_t server_head3(const float* P2, int S2, int64_t slab2, Epi e2, const float* W3, const float* b3,
                        const int64_t* y, int64_t ignore, float scale, float* h2, float* dlog, float* dz2,
                        float* loss_rows, int M, int N2, int C, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  const size_t shmem = (size_t)(((N2 + 3) & ~3) + C) * sizeof(float);
  // column slices of <= 64 float4 so phase 4 has >= 4 output groups per column
  const int n4 = N2 / 4;
  const int Q = max(1, (n4 + 63) / 64);
  head3_kernel<<<dim3(M, Q), 256, shmem, st>>>(P2, S2, slab2, e2, W3, b3, y, ignore, scale, h2, dlog, dz2, loss_rows,
                                               N2, C);
  return hipGetLastError();
}

hipError_t wgrad_group(const WgGroup& g, int M, SlOpt o, hipStream_t st) {
  int kmax = 0, yb = 0;
  WgGroup gg = g;
  for (int i = 0; i < gg.n; ++i) {
    gg.d[i].yb0 = yb;
    yb += (gg.d[i].N + 15) / 16;
    kmax = max(kmax, gg.d[i].K);
  }
  if (yb == 0 || kmax == 0) return hipSuccess;
  dim3 grid((kmax + 255) / 256, yb);
  if (o.kind == 2)
    wgrad_group_kernel<true><<<grid, 1024, 0, st>>>(gg, M, o);
  else
    wgrad_group_kernel<false><<<grid, 1024, 0, st>>>(gg, M, o);
  return hipGetLastError();
}

}  // namespace sl
