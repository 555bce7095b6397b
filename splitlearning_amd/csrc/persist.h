// Device helpers shared by the persistent server-epoch kernels (csrc/resident.hip,
// csrc/hybrid.hip): hand-off loads / stores through buffer resources (write-through sc1
// stores, L1-bypassing sc1 loads: MI355X_MICROARCH.md, the valid-forms table row 1), relaxed
// counter polls, the dropout epilogue and the optimizer update with per-step scalars in VGPRs.
#pragma once
#include "common.h"

namespace sl {
namespace persist {

typedef int res_i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
// hand-off traffic: write-through (sc1) stores and L1-bypassing (sc1) loads (aux 16)
__device__ __forceinline__ f32x4 hld4(__amdgpu_buffer_rsrc_t rs, int boff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 16));
}
__device__ __forceinline__ float hld1(__amdgpu_buffer_rsrc_t rs, int boff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, boff, 0, 16));
}
__device__ __forceinline__ void hst4(__amdgpu_buffer_rsrc_t rs, int boff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, v), rs, boff, 0, 16);
}
__device__ __forceinline__ void hst1(__amdgpu_buffer_rsrc_t rs, int boff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rs, boff, 0, 16);
}

__device__ __forceinline__ unsigned poll(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool failed(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

__device__ __forceinline__ float drop_relu(float v, uint32_t lo, uint32_t hi, uint32_t row, uint32_t col,
                                           uint32_t thr, float dsc) {
  v = fmaxf(v, 0.f);
  if (thr) v = sl_hash_keep(lo, hi, row, col, thr) ? v * dsc : 0.f;
  return v;
}

// The optimizer step of one element: sl_opt_update's arithmetic (common.h) for SGD-momentum /
// Adam, with the step's Adam scalars passed in VGPRs (ss = lr / (1 - beta1^t), ib = 1 /
// sqrt(1 - beta2^t); as SGPR operands they pushed the kernel's scalar registers into spills)
// and the hardware square root and reciprocal (v_sqrt_f32 / v_rcp_f32, 1 ulp) in place of the
// correctly rounded sqrtf and division: with the state on-chip the update is VALU-bound (a TP
// = 8 shard's 16 K elements per CU took 4-5 us of the step with the IEEE sequences, ~25
// instructions each), and 1 ulp of the update is ~1e-10 absolute at lr 1e-3, far inside the
// torch comparison (tests/test_resident_gpu.py).
template <bool ADAM>
__device__ __forceinline__ void res_update(const SlOpt& o, float ss, float ib, float& p, float g, float& s0,
                                           float& s1) {
  if (o.wd != 0.f) g = fmaf(o.wd, p, g);
  if (!ADAM) {
    const float b = (o.momentum != 0.f) ? fmaf(o.momentum, s0, g) : g;
    s0 = b;
    p = fmaf(-o.lr, b, p);
  } else {
    const float m = fmaf(o.beta1, s0, (1.f - o.beta1) * g);
    const float v = fmaf(o.beta2, s1, (1.f - o.beta2) * g * g);
    s0 = m;
    s1 = v;
    const float denom = __builtin_amdgcn_sqrtf(v) * ib + o.eps;
    p = p - ss * (m * __builtin_amdgcn_rcpf(denom));
  }
}
// Four elements as two packed pairs (v_pk_fma_f32 / v_pk_mul_f32; the square root and the
// reciprocal per element): the same operations as res_update, half the VALU issue slots.
typedef float res_f32x2 __attribute__((ext_vector_type(2)));
template <bool ADAM>
__device__ __forceinline__ void res_update2(const SlOpt& o, float ss, float ib, res_f32x2& p, res_f32x2 g,
                                            res_f32x2& s0, res_f32x2& s1) {
  if (o.wd != 0.f) g = __builtin_elementwise_fma(res_f32x2{o.wd, o.wd}, p, g);
  if (!ADAM) {
    const res_f32x2 b = (o.momentum != 0.f) ? __builtin_elementwise_fma(res_f32x2{o.momentum, o.momentum}, s0, g) : g;
    s0 = b;
    p = __builtin_elementwise_fma(res_f32x2{-o.lr, -o.lr}, b, p);
  } else {
    const float c1 = 1.f - o.beta1, c2 = 1.f - o.beta2;
    const res_f32x2 m = __builtin_elementwise_fma(res_f32x2{o.beta1, o.beta1}, s0, res_f32x2{c1, c1} * g);
    const res_f32x2 v = __builtin_elementwise_fma(res_f32x2{o.beta2, o.beta2}, s1, (res_f32x2{c2, c2} * g) * g);
    s0 = m;
    s1 = v;
    const res_f32x2 sq = {__builtin_amdgcn_sqrtf(v[0]), __builtin_amdgcn_sqrtf(v[1])};
    const res_f32x2 den = __builtin_elementwise_fma(sq, res_f32x2{ib, ib}, res_f32x2{o.eps, o.eps});
    const res_f32x2 rc = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
    p = p - res_f32x2{ss, ss} * (m * rc);
  }
}
template <bool ADAM>
__device__ __forceinline__ void res_update4(const SlOpt& o, float ss, float ib, f32x4& p, f32x4 g, f32x4& s0,
                                            f32x4& s1) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    res_f32x2 pp = {p[2 * h], p[2 * h + 1]}, a0 = {s0[2 * h], s0[2 * h + 1]}, a1 = {s1[2 * h], s1[2 * h + 1]};
    res_update2<ADAM>(o, ss, ib, pp, res_f32x2{g[2 * h], g[2 * h + 1]}, a0, a1);
    p[2 * h] = pp[0];
    p[2 * h + 1] = pp[1];
    s0[2 * h] = a0[0];
    s0[2 * h + 1] = a0[1];
    s1[2 * h] = a1[0];
    s1[2 * h + 1] = a1[1];
  }
}

}  // namespace persist
}  // namespace sl
