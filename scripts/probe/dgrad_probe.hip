// Standalone timing probe of fc2's data gradient (dz1 = dz2 . W2, masked) at the server-step
// shape (M 16, N 1000, K 5000; and the TP = 8 shard K = 628): the package's split-N kernel +
// reduce against launch-geometry variants, GPU time per launch from graph replay (hot / warm
// = behind a 48 MB memset / cold = behind a 512 MB memset).  Not part of the package.
#include "../../splitlearning_amd/csrc/linear.hip"
#include "../../splitlearning_amd/csrc/fused.hip"
#include "../../splitlearning_amd/csrc/gemm.hip"

#include <cstdio>
#include <functional>
#include <vector>

using namespace sl;

static hipStream_t g_s = 0;

// float4-vectorised reduce of S split-N slabs + mask (dgrad_reduce_kernel does one float per thread)
__global__ void dgrad_reduce4_kernel(const float* __restrict__ P, int S, int64_t slab, const float* __restrict__ hprev,
                                     float scale, float* __restrict__ out, int64_t n4) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n4) return;
  const f32x4* p = reinterpret_cast<const f32x4*>(P) + t;
  f32x4 r[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) r[s] = s < S ? p[s * (slab >> 2)] : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) v += r[s];
  const f32x4 h = reinterpret_cast<const f32x4*>(hprev)[t];
  f32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = h[i] > 0.f ? v[i] * scale : 0.f;
  reinterpret_cast<f32x4*>(out)[t] = o;
}

template <class F>
static float graph_us(F f, int n, int reps, void* flush, size_t fbytes, bool cold) {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  g_s = s;
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
  const int M = 16, N = 1000;
  void* flush;
  const size_t fbytes = 512ull << 20;
  if (hipMalloc(&flush, fbytes) != hipSuccess) return 1;
  for (int K : {5000, 628}) {
    float *W, *dz, *h, *ws, *out;
    (void)hipMalloc(&W, sizeof(float) * N * K);
    (void)hipMalloc(&dz, sizeof(float) * M * N);
    (void)hipMalloc(&h, sizeof(float) * M * K);
    (void)hipMalloc(&ws, sizeof(float) * 64 * M * K);
    (void)hipMalloc(&out, sizeof(float) * M * K);
    (void)hipMemset(W, 0, sizeof(float) * N * K);
    (void)hipMemset(dz, 0, sizeof(float) * M * N);
    (void)hipMemset(h, 0, sizeof(float) * M * K);
    const int kt = (K + 63) / 64;
    const int64_t slab = (int64_t)M * K;
    auto dg = [&](int S, int nw) {
      return [=] {
        if (nw == 8)
          skinny_dgrad_kernel<8><<<dim3(kt, 1, S), 512, 0, g_s>>>(dz, N, W, K, nullptr, 0, 1.f, ws, 0, slab, M, N, K);
        else if (nw == 4)
          skinny_dgrad_kernel<4><<<dim3(kt, 1, S), 256, 0, g_s>>>(dz, N, W, K, nullptr, 0, 1.f, ws, 0, slab, M, N, K);
        else
          skinny_dgrad_kernel<16><<<dim3(kt, 1, S), 1024, 0, g_s>>>(dz, N, W, K, nullptr, 0, 1.f, ws, 0, slab, M, N, K);
      };
    };
    auto red = [=](int S) {
      return [=] {
        dgrad_reduce_kernel<<<(unsigned)((M * K + 255) / 256), 256, 0, g_s>>>(ws, S, slab, h, K, 2.f, out, K, M, K);
      };
    };
    auto red4 = [=](int S) {
      return [=] {
        const int64_t n4 = (int64_t)M * K / 4;
        dgrad_reduce4_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, g_s>>>(ws, S, slab, h, 2.f, out, n4);
      };
    };
    auto pair = [](std::function<void()> a, std::function<void()> b) {
      return [=] {
        a();
        b();
      };
    };
    struct Row {
      std::string name;
      std::function<void()> f;
    };
    std::vector<Row> rows;
    for (int S : {4, 8, 16, 32}) {
      for (int nw : {4, 8, 16}) {
        if ((N + 4 * S - 1) / (4 * S) * 4 < 4 * nw) continue;      // every wave gets >= 4 rows
        char b[96];
        snprintf(b, sizeof b, "dgrad S %2d waves %2d", S, nw);
        rows.push_back({b, dg(S, nw)});
      }
      char b[96];
      snprintf(b, sizeof b, "reduce S %2d (scalar)", S);
      rows.push_back({b, red(S)});
      snprintf(b, sizeof b, "reduce S %2d (float4)", S);
      rows.push_back({b, red4(S)});
      snprintf(b, sizeof b, "dgrad S %2d w8 + reduce", S);
      rows.push_back({b, pair(dg(S, 8), red(S))});
      snprintf(b, sizeof b, "dgrad S %2d w8 + reduce4", S);
      rows.push_back({b, pair(dg(S, 8), red4(S))});
    }
    printf("K = %d (%d k tiles)\n", K, kt);
    for (auto& r : rows) {
      const float hot = graph_us(r.f, 50, 20, flush, fbytes, false);
      const size_t wb = 48ull << 20;
      const float warm = graph_us(r.f, 20, 5, flush, wb, true) - graph_us([] {}, 20, 5, flush, wb, true);
      const float cold = graph_us(r.f, 20, 5, flush, fbytes, true) - graph_us([] {}, 20, 5, flush, fbytes, true);
      printf("  %-28s hot %7.2f   warm %7.2f   cold %7.2f  us\n", r.name.c_str(), hot, warm, cold);
    }
    (void)hipFree(W);
    (void)hipFree(dz);
    (void)hipFree(h);
    (void)hipFree(ws);
    (void)hipFree(out);
  }
  (void)hipDeviceSynchronize();
  return 0;
}
