// Fused U-shape middle + head: one launch per batch of the co-located U-shape split epoch
// (csrc/split.cpp SplitEpoch::bob_ushape) in place of three -- the fc1 look-ahead epilogue
// (linear_epilogue), the fc2 forward (skinny_fwd_once_kernel<4>) and Alice's head step
// (head_step_mfma_kernel).  Reference hot loop: data_entities.py:65-81 (Bob's model2 forward,
// Alice's model3 + CrossEntropyLoss, the backward and both optimizer steps).
//
// Grid: J = ceil(N1 / 64) workgroups of 256 threads.  Workgroup j owns h1 columns
// [64 j, 64 j + 64): it forms them (the S look-ahead slabs summed in slab order + b1, ReLU:
// epilogue_kernel's arithmetic), stores them (the fc2 dgrad mask and fc2 wgrad operand), and
// forms the fc2 partial of that k-range for every 16-column tile exactly as wave j of
// skinny_fwd_once_kernel<4> does (same operands, same MFMA order).  It stores the partials
// write-through and arrives on a counter; the LAST arriver (no workgroup ever waits) sums the
// J partials in wave order -- that kernel's reduction -- applies fc2's epilogue, and runs the
// head step on h2 straight from LDS (head_core.h).  The results are the three launches' bits:
// tests/test_split_native_gpu.py holds the native epoch bitwise to the Python loop, which
// still issues the three launches.
#include "common.h"
#include "head_core.h"
#include "persist.h"
#include "ushape.h"

namespace sl {

extern int g_bf16;

namespace {

constexpr int kMidThreads = 256;
constexpr int kMidMaxJ = 16;     // skinny_fwd_once_kernel runs unsplit up to 16 waves (N1 <= 1024)
constexpr int PHB = 68;          // h1 block row pitch (floats)

__device__ __forceinline__ f32x4 mid_mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

}  // namespace

__global__ void __launch_bounds__(kMidThreads) ushape_mid_kernel(MidArgs a) {
  __shared__ __attribute__((aligned(16))) HeadLds L;
  __shared__ int s_last;
  const int j = blockIdx.x, J = gridDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = a.M, N1 = a.N1, N2 = a.N2, NT = (N2 + 15) >> 4;
  const int k0 = 64 * j;
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rP = persist::rs_of(a.part);

  // ---- h1 columns [k0, k0 + 64) into hb [16][PHB] (L.sg's space, free until the head)
  float* hb = &L.sg[0][0];
  {
    const int m = tid >> 4, q = 4 * (tid & 15), n = k0 + q;
    f32x4 v = zv;
    if (m < M && n < N1) {   // N1 % 4 == 0: a float4 never straddles N1
      if (a.pn != nullptr) {
        // sum_slabs (common.h) on four columns: 32 slabs per round, zeros past S, slab order
        const float* p = a.pn + (int64_t)m * N1 + n;
        f32x4 acc = zv;
        for (int s0 = 0; s0 < a.S; s0 += 32) {
          f32x4 r[32];
#pragma unroll
          for (int i = 0; i < 32; ++i)
            r[i] = (s0 + i < a.S) ? *reinterpret_cast<const f32x4*>(p + (int64_t)(s0 + i) * a.slab) : zv;
#pragma unroll
          for (int i = 0; i < 32; ++i) acc += r[i];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = apply_epi(a.e1, acc[c], m, n + c);
        *reinterpret_cast<f32x4*>(a.h1 + (int64_t)m * N1 + n) = v;
      } else {
        v = *reinterpret_cast<const f32x4*>(a.h1 + (int64_t)m * N1 + n);
      }
    }
    *reinterpret_cast<f32x4*>(hb + m * PHB + q) = v;
  }
  __syncthreads();

  // ---- fc2 partial over k in [k0, k0 + 64) per 16-column tile: wave j of
  // skinny_fwd_once_kernel<4> (linear.hip), operand for operand
  {
    const int ra = lane & 15, kq = (lane >> 4) * 4;
    for (int bx = wv; bx < NT; bx += 4) {
      const int rb = 16 * bx + (lane & 15);
      const bool vb = rb < N2;
      const float* pb = a.W2 + (int64_t)(vb ? rb : 0) * N1;
      f32x4 av[4], w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k0 + 16 * u + kq;
        const bool in = kk < N1;
        av[u] = in ? *reinterpret_cast<const f32x4*>(hb + ra * PHB + 16 * u + kq) : zv;
        w[u] = (vb && in) ? *reinterpret_cast<const f32x4*>(pb + kk) : zv;
      }
      f32x4 acc0 = zv, acc1 = zv;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc0 = mid_mfma4(av[u][0], w[u][0], acc0);
        acc1 = mid_mfma4(av[u][1], w[u][1], acc1);
        acc0 = mid_mfma4(av[u][2], w[u][2], acc0);
        acc1 = mid_mfma4(av[u][3], w[u][3], acc1);
      }
      persist::hst4(rP, ((j * NT + bx) * 64 + lane) * 16, acc0 + acc1);
    }
  }

  // ---- the head's operands that need no h2, in flight while this workgroup arrives (whichever
  // workgroup is last runs the head)
  HeadPre P;
  head_preload(P, a.hw, a.hb, a.s0w, a.s1w, a.s0b, a.s1b, N2, a.C);

  // ---- arrive (every wave drained its write-through stores first); the last one goes on
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old + 1 == (unsigned)J;
    if (last) __hip_atomic_store(a.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;

  // ---- h2 = epilogue(the J partials summed in wave order) -> global and the head's X
  for (int i = tid; i < 16 * HeadLds::KP; i += kMidThreads) (&L.sx[0][0])[i] = 0.f;
  __syncthreads();
  for (int bx = wv; bx < NT; bx += 4) {
    f32x4 p[kMidMaxJ];
#pragma unroll
    for (int i = 0; i < kMidMaxJ; ++i) p[i] = i < J ? persist::hld4(rP, ((i * NT + bx) * 64 + lane) * 16) : zv;
    f32x4 s = p[0];
#pragma unroll
    for (int i = 1; i < kMidMaxJ; ++i)
      if (i < J) s += p[i];
    const int n = 16 * bx + (lane & 15);
    if (n < N2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (lane >> 4) * 4 + r;
        if (m < M) {
          const float v = apply_epi(a.e2, s[r], m, n);
          a.h2[m * N2 + n] = v;
          L.sx[m][n] = v;
        }
      }
    }
  }
  __syncthreads();
  head_core<false>(L, P, true, a.h2, a.hb, a.y, a.ignore, a.scale, a.loss_rows, a.dz2, a.hw, a.hb, a.s0w, a.s1w,
                   a.s0b, a.s1b, M, N2, a.C, a.o, 1);
}

// Whether the fused launch covers this shape (fp32; otherwise the three launches run).
bool ushape_mid_ok(int M, int N1, int N2, int C) {
  const int J = (N1 + 63) / 64;
  return g_bf16 == 0 && M >= 1 && M <= 16 && J >= 1 && J <= kMidMaxJ && (N1 & 3) == 0 && N2 >= 4 && N2 <= 128 &&
         (N2 & 3) == 0 && C >= 1 && C <= 16 && C * N2 <= 2048;
}

// partial workspace in floats for N1, N2
int64_t ushape_mid_part_floats(int N1, int N2) {
  return (int64_t)((N1 + 63) / 64) * ((N2 + 15) / 16) * 64 * 4;
}

hipError_t ushape_mid(const MidArgs& a, hipStream_t st) {
  if (!ushape_mid_ok(a.M, a.N1, a.N2, a.C)) return hipErrorInvalidValue;
  if (((reinterpret_cast<uintptr_t>(a.h1) | reinterpret_cast<uintptr_t>(a.W2) | reinterpret_cast<uintptr_t>(a.hw) |
        reinterpret_cast<uintptr_t>(a.part) | reinterpret_cast<uintptr_t>(a.pn)) & 15) != 0)
    return hipErrorInvalidValue;
  ushape_mid_kernel<<<(a.N1 + 63) / 64, kMidThreads, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace sl
