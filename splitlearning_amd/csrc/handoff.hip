// Hand-off stress test: the persistent kernels' in-launch publication primitive, checked word
// by word under uneven load (MI355X_MICROARCH.md: "test every hand-off under UNEVEN load,
// consumer L1-warm, checking every word").
//
// Why: csrc/resident.hip, hybrid.hip and vanilla.hip hand tiles between workgroups inside one
// launch with the valid-forms table's row 1 (persist.h): the producer stores the payload
// write-through (sc1), every wave drains (`s_waitcnt vmcnt(0)`), a workgroup barrier, then
// ONE lane adds to a per-XCD counter shard (relaxed, agent scope); the consumer polls the
// shards (relaxed agent loads = `sc1` loads), a workgroup barrier releases its waves, and
// every load of the payload is an `sc1` buffer load (L1 bypassed).  This kernel runs exactly
// that primitive (persist.h's own hst4 / hld4 / poll) in the harshest pattern the kernels
// have: a payload REWRITTEN IN PLACE every round (as vanilla's fc1 tiles are between its
// update and forward passes), consumers that re-read the same addresses every round (L1 and
// L2 warm with the previous round's value), producers on every XCD, and per-round random
// delays plus a bandwidth stream on a random subset of workgroups.  A second seam ("reads
// done") gates the next round's rewrite, as the kernels' seam chains do.
//
// Modes (what the host asks for; tests/test_handoff_gpu.py):
//   0  shipped: sc1 stores + drained counter add; sc1 loads after the poll
//   1  negative control: plain stores, plain loads, no fences (stale reads expected)
//   2  sc1 stores, plain loads (L1 may serve a stale line: expected stale)
//   3  the LLVM AMDGPU memory model's own form: plain stores, agent RELEASE fence before the
//      counter add; agent ACQUIRE fence after the poll, plain loads
//   4  shipped + agent acquire after the poll (belt and braces)
// Every wait is bounded (wall clock): a timeout raises err and every later wait gives up, so
// the grid always drains.
#include "handoff.h"
#include "persist.h"

namespace sl {

namespace {

using namespace persist;

__device__ __forceinline__ uint32_t ho_val(uint32_t r, uint32_t src, uint32_t idx) {
  return sl_fmix32((r * 0x9E3779B1u) ^ (src * 0x85EBCA77u) ^ (idx * 0xC2B2AE3Du));
}

__device__ __forceinline__ bool ho_wait(const HoArgs& a, int seam, unsigned tgt, int* s_ok) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < 8) {
      const unsigned* p = a.cnt + (seam * 8 + lane) * kHoStride;
      if (poll(p) < tgt) {
        const uint64_t t0 = wall_clock64();
        while (poll(p) < tgt) {
          if (failed(a.err)) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if ((int64_t)(wall_clock64() - t0) > a.timeout) {
            __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = false;
            break;
          }
        }
      }
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return *s_ok != 0;
}

template <int MODE>
__global__ void __launch_bounds__(kHoThreads) handoff_stress_kernel(HoArgs a) {
  __shared__ int s_ok;
  __shared__ unsigned s_bad[kHoThreads / 64];
  const int w = blockIdx.x, G = gridDim.x, tid = threadIdx.x;
  const int P4 = a.P >> 2;   // float4 per payload
  const __amdgpu_buffer_rsrc_t rD = rs_of(a.D);
  const __amdgpu_buffer_rsrc_t rS = rs_of(a.scratch);
  const unsigned per = (unsigned)(G / 8);   // arrivals per shard and round
  unsigned bad = 0;
  for (int r = 1; r <= a.R; ++r) {
    // the previous round's reads are done everywhere before this payload is rewritten
    if (r > 1 && !ho_wait(a, 1, per * (unsigned)(r - 1), &s_ok)) break;
    // uneven load: a random delay, and on a random half of the workgroups a read-modify-write
    // stream over this workgroup's 64 KB of scratch (plain accesses: L2 / fabric pressure)
    const uint32_t hz = sl_fmix32((uint32_t)r * 0x27d4eb2du ^ (uint32_t)w * 0x165667b1u);
    if (hz & 1u) {
      for (int e = tid; e < kHoScratchF4; e += kHoThreads) {
        const int off = ((w * kHoScratchF4) + e) * 16;
        f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rS, off, 0, 0));
        v += 1.f;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, v), rS, off, 0, 0);
      }
    }
    if (a.busy_ticks > 0) {
      const uint64_t t0 = wall_clock64(), dt = (hz >> 8) % (uint32_t)a.busy_ticks;
      while (wall_clock64() - t0 < dt) __builtin_amdgcn_s_sleep(1);
    }
    // produce
    for (int e = tid; e < P4; e += kHoThreads) {
      res_i32x4 v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = (int)ho_val((uint32_t)r, (uint32_t)w, (uint32_t)(4 * e + c));
      const int off = (w * P4 + e) * 16;
      if (MODE == 0 || MODE == 2 || MODE == 4)
        __builtin_amdgcn_raw_buffer_store_b128(v, rD, off, 0, 16);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, rD, off, 0, 0);
    }
    // publish: every wave drains, barrier, one lane adds (MODE 3: behind an agent release)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      if (MODE == 3) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_fetch_add(a.cnt + (0 * 8 + (w & 7)) * kHoStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!ho_wait(a, 0, per * (unsigned)r, &s_ok)) break;
    if (MODE == 3 || MODE == 4) {
      if (tid < 64) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
    // consume: nsrc producers (same XCD and other XCDs), every word checked
    for (int s = 0; s < a.nsrc; ++s) {
      const int src = (w + 1 + s * a.src_stride) % G;
      for (int e = tid; e < P4; e += kHoThreads) {
        const int off = (src * P4 + e) * 16;
        const res_i32x4 v = (MODE == 0 || MODE == 4) ? __builtin_amdgcn_raw_buffer_load_b128(rD, off, 0, 16)
                                                      : __builtin_amdgcn_raw_buffer_load_b128(rD, off, 0, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t want = ho_val((uint32_t)r, (uint32_t)src, (uint32_t)(4 * e + c));
          if ((uint32_t)v[c] != want) {
            ++bad;
            if (a.first[0] == 0u &&
                __hip_atomic_fetch_add(a.first, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
              a.first[1] = (unsigned)r;
              a.first[2] = (unsigned)src;
              a.first[3] = (unsigned)(4 * e + c);
              a.first[4] = (uint32_t)v[c];
              a.first[5] = want;
              a.first[6] = (unsigned)w;
            }
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(a.cnt + (1 * 8 + (w & 7)) * kHoStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) a.done[w] = (unsigned)r;
  }
  // per-workgroup mismatch count
  bad += __shfl_xor(bad, 1);
  bad += __shfl_xor(bad, 2);
  bad += __shfl_xor(bad, 4);
  bad += __shfl_xor(bad, 8);
  bad += __shfl_xor(bad, 16);
  bad += __shfl_xor(bad, 32);
  if ((tid & 63) == 0) s_bad[tid >> 6] = bad;
  __syncthreads();
  if (tid == 0) {
    unsigned t = 0;
    for (int i = 0; i < kHoThreads / 64; ++i) t += s_bad[i];
    a.bad[w] = t;
  }
}

}  // namespace

std::string handoff_check(const HoArgs& a, int G) {
  if (G < 8 || G > 1024 || G % 8) return "workgroups: a multiple of 8, 8..1024";
  if (a.P < 4 || a.P % 4 || (int64_t)G * a.P > (1LL << 27)) return "payload words";
  if (a.nsrc < 1 || a.nsrc > 16 || a.src_stride < 1) return "sources";
  if (a.R < 1 || a.mode < 0 || a.mode > 4) return "rounds / mode";
  return "";
}

hipError_t handoff_stress_launch(const HoArgs& a, int G, hipStream_t st) {
  if (!handoff_check(a, G).empty()) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.cnt, 0, (size_t)2 * 8 * kHoStride * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  void* params[] = {const_cast<HoArgs*>(&a)};
  const void* fn = nullptr;
  switch (a.mode) {
    case 0: fn = reinterpret_cast<const void*>(&handoff_stress_kernel<0>); break;
    case 1: fn = reinterpret_cast<const void*>(&handoff_stress_kernel<1>); break;
    case 2: fn = reinterpret_cast<const void*>(&handoff_stress_kernel<2>); break;
    case 3: fn = reinterpret_cast<const void*>(&handoff_stress_kernel<3>); break;
    default: fn = reinterpret_cast<const void*>(&handoff_stress_kernel<4>); break;
  }
  // cooperative: every workgroup waits on every other one, so all must be resident at once
  return hipLaunchCooperativeKernel(fn, dim3(G), dim3(kHoThreads), params, 0, st);
}

}  // namespace sl
