// Shared device helpers for the splitlearning_amd gfx950 kernels.
//
// Everything here is CDNA4-native: wave64 reductions, counter-based dropout
// hash (bit-identical to ops/rng.py), and the fused optimizer update used by
// every "gradient + step" kernel (torch.optim.SGD / Adam semantics, see
// ops/torch_ops.py::adam_update_ / sgd_update_).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SL_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ RNG
__device__ __forceinline__ uint32_t sl_fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}
// keep iff hash >= thresh, thresh = p * 2^32 (host computes it).
__device__ __forceinline__ bool sl_hash_keep(uint32_t seed_lo, uint32_t seed_hi, uint32_t row,
                                             uint32_t col, uint32_t thresh) {
  uint32_t a = sl_fmix32((row * 0x9E3779B1u) ^ seed_lo);
  uint32_t h = sl_fmix32(a ^ ((col * 0x85EBCA77u) ^ seed_hi));
  return h >= thresh;
}

// ------------------------------------------------------------------ bf16 compute
// `--dtype bf16`: a GEMM operand rounded to bf16 (RNE; v_cvt_pk_bf16_f32) and back.  The
// product of two such values is exact in fp32, so rounding the operands and accumulating in
// fp32 has the numerics of a bf16 MFMA with fp32 accumulation (up to summation order); the
// memory-bound skinny kernels use this form, the compute-bound ones the bf16 MFMA itself.
__device__ __forceinline__ float bfr(float x) { return (float)(__bf16)x; }
__device__ __forceinline__ f32x4 bfr4(f32x4 v) { return f32x4{bfr(v[0]), bfr(v[1]), bfr(v[2]), bfr(v[3])}; }
__device__ __forceinline__ float4 bfr4(float4 v) { return make_float4(bfr(v.x), bfr(v.y), bfr(v.z), bfr(v.w)); }

// ------------------------------------------------------------------ reductions

// Row (16-lane) reductions on DPP lane moves instead of LDS-routed ds_bpermute shuffles:
// xor 1 and xor 2 (quad_perm), then row_half_mirror (lane i <-> 7 - i) and row_mirror (lane
// i <-> 15 - i).  Every lane of a row ends with the same, bitwise identical total.  A wave
// total is the four row totals read with v_readlane (sl_wave_sum_dpp / sl_wave_max_dpp).
template <int CTRL>
__device__ __forceinline__ float sl_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sl_row16_sum(float v) {
  v += sl_dpp<0xB1>(v);
  v += sl_dpp<0x4E>(v);
  v += sl_dpp<0x141>(v);
  v += sl_dpp<0x140>(v);
  return v;
}
__device__ __forceinline__ float sl_row16_max(float v) {
  v = fmaxf(v, sl_dpp<0xB1>(v));
  v = fmaxf(v, sl_dpp<0x4E>(v));
  v = fmaxf(v, sl_dpp<0x141>(v));
  v = fmaxf(v, sl_dpp<0x140>(v));
  return v;
}
// value of lane (row base + j) of this lane's 16-lane row (j uniform within the row or not:
// ds_bpermute-free via a DPP-built row, here simply a bpermute inside the row)
__device__ __forceinline__ float sl_dpp_pick(float v, int j) {
  const int src = ((int)(__lane_id()) & ~15) + (j & 15);
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src << 2, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float sl_lane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float sl_wave_sum_dpp(float v) {
  v = sl_row16_sum(v);
  return (sl_lane(v, 0) + sl_lane(v, 16)) + (sl_lane(v, 32) + sl_lane(v, 48));
}
__device__ __forceinline__ float sl_wave_max_dpp(float v) {
  v = sl_row16_max(v);
  return fmaxf(fmaxf(sl_lane(v, 0), sl_lane(v, 16)), fmaxf(sl_lane(v, 32), sl_lane(v, 48)));
}
// Whole-wave sum / max, returned to every lane.  Call with all 64 lanes active.
__device__ __forceinline__ float sl_wave_sum(float v) { return sl_wave_sum_dpp(v); }
__device__ __forceinline__ float sl_wave_max(float v) { return sl_wave_max_dpp(v); }
// Sum over aligned groups of SUB consecutive lanes (SUB a power of two <= 64), returned to
// every lane of the group: DPP moves inside a 16-lane row, ds_bpermute across rows.
template <int SUB>
__device__ __forceinline__ float sl_group_sum(float v) {
  if (SUB >= 2) v += sl_dpp<0xB1>(v);
  if (SUB >= 4) v += sl_dpp<0x4E>(v);
  if (SUB >= 8) v += sl_dpp<0x141>(v);
  if (SUB >= 16) v += sl_dpp<0x140>(v);
  if (SUB >= 32) v += __shfl_xor(v, 16, 64);
  if (SUB >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}

// ------------------------------------------------------------------ partial-sum slabs
// Sum of S split-K / split-N partials p[0], p[slab], ...: up to 32 slabs are loaded with
// every load issued before the first add (one memory round trip instead of S / 4), in
// slab order so the result is bit-identical to the sequential sum.
__device__ __forceinline__ float sum_slabs(const float* __restrict__ p, int S, int64_t slab) {
  constexpr int U = 32;
  float v = 0.f;
  int s0 = 0;
  for (; s0 < S; s0 += U) {
    float r[U];
#pragma unroll
    for (int i = 0; i < U; ++i) r[i] = (s0 + i < S) ? p[(int64_t)(s0 + i) * slab] : 0.f;
#pragma unroll
    for (int i = 0; i < U; ++i) v += r[i];
  }
  return v;
}

// ------------------------------------------------------------------ optimizer
// kind: 0 = write gradient only (p untouched, grad -> s0), 1 = SGD(momentum), 2 = Adam (L2 wd).
struct SlOpt {
  int kind;
  float lr;
  float beta1, beta2, eps, wd, momentum;
  float step_size;     // Adam: lr / (1 - beta1^t)
  float inv_bc2_sqrt;  // Adam: 1 / sqrt(1 - beta2^t)
  // graph replay: when set, {step_size, inv_bc2_sqrt} are read from device memory so a
  // captured step can be replayed at any step count (the host refreshes the table).
  const float* dyn;
};

// Update one element. s0 = m (Adam) / momentum buffer (SGD) / grad out (kind 0); s1 = v (Adam).
__device__ __forceinline__ void sl_opt_update(const SlOpt& o, float& p, float g, float& s0, float& s1) {
  if (o.kind == 0) { s0 = g; return; }
  if (o.wd != 0.f) g = fmaf(o.wd, p, g);
  if (o.kind == 1) {
    float b = (o.momentum != 0.f) ? fmaf(o.momentum, s0, g) : g;
    s0 = b;
    p = fmaf(-o.lr, b, p);
  } else {
    float m = fmaf(o.beta1, s0, (1.f - o.beta1) * g);
    float v = fmaf(o.beta2, s1, (1.f - o.beta2) * g * g);
    s0 = m; s1 = v;
    const float ss = o.dyn ? o.dyn[0] : o.step_size;
    const float ib = o.dyn ? o.dyn[1] : o.inv_bc2_sqrt;
    float denom = sqrtf(v) * ib + o.eps;
    p = p - ss * (m / denom);
  }
}

// A client optimizer step not yet stored (split modes, conv.hip): the B partial dW/db slabs
// of the last backward and that step's optimizer scalars.  The next forward applies it for
// its own use and the next backward stores it (FrontEngine's deferred update).
struct ConvPending {
  const float* slab;
  int B;
  float* s0w;
  float* s1w;
  float* s0b;
  float* s1b;
  SlOpt o;
};

// One co-located Alice's frozen-front forward, for conv_fwd_multi (conv.hip): rows
// idx[0 .. n) (or 0 .. n when idx is null) of her uint8 shard x -> y [n, 5408].
struct FrontFwdDesc {
  const uint8_t* x;
  const int64_t* idx;
  int64_t n;
  const float* w;
  const float* b;
  float* y;
};
constexpr int kFrontFwdMax = 16;
struct FrontFwdSet {
  FrontFwdDesc d[kFrontFwdMax];
  int k;
};

// One co-located Alice's local epoch, for conv_local_epoch_multi (conv.hip).
struct MultiAlice {
  const uint8_t* x;        // shard pixels [N, 784]
  const int64_t* order;    // this epoch's sample order [n]
  int64_t n;
  const int64_t* labels;   // shard labels [N]
  float *w, *b, *s0w, *s1w, *s0b, *s1b;
  float* ws;               // >= 2 B 320 + 2 960 floats, private to this Alice
  int64_t ws_elems;
  float* loss_rows;        // [n]
  int64_t t0;              // first optimizer step of the epoch
};

// Fused GEMM epilogue: bias, ReLU, counter-hash dropout (global column index).
struct Epi {
  const float* bias;
  int relu;
  uint32_t thresh;      // dropout keep iff hash >= thresh (0 = no dropout)
  float dscale;         // 1/(1-p)
  uint32_t seed_lo, seed_hi;
  int col_off;          // global column index of column 0 (tensor-parallel shards)
  const uint32_t* dseed;  // graph replay: {seed_lo, seed_hi} from device memory when set
};

__device__ __forceinline__ float apply_epi(const Epi& e, float v, int m, int n) {
  if (e.bias) v += e.bias[n];
  if (e.relu) v = fmaxf(v, 0.f);
  if (e.thresh) {
    const uint32_t lo = e.dseed ? e.dseed[0] : e.seed_lo, hi = e.dseed ? e.dseed[1] : e.seed_hi;
    v = sl_hash_keep(lo, hi, (uint32_t)m, (uint32_t)(e.col_off + n), e.thresh) ? v * e.dscale : 0.f;
  }
  return v;
}

// Vector form of sl_opt_update (the f32x4 elements cannot bind to float&).
template <bool ADAM>
__device__ __forceinline__ void sl_opt_update4(const SlOpt& o, f32x4& p, f32x4 g, f32x4& s0, f32x4& s1) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float pp = p[i], a0 = s0[i], a1 = ADAM ? s1[i] : 0.f;
    sl_opt_update(o, pp, g[i], a0, a1);
    p[i] = pp;
    s0[i] = a0;
    if (ADAM) s1[i] = a1;
  }
}

// Kernel-variant switches for in-process A/B measurement (set from Python via
// _C.set_variant; 0 = the shipped default everywhere).
namespace sl {
extern int g_variant[24];

extern int g_bf16;      // compute dtype of the GEMM-shaped kernels: 0 = exact fp32, 1 = bf16 operands
extern int g_nn_splits;  // gemm_nn_dgrad's reduction split: 0 = its own choice, else forced (A/B sweeps)
extern int g_nn_wm;      // gemm_nn_dgrad's tile form: 0 = its own choice, 2 / 4 forced (A/B sweeps)
extern int g_nt_splits;  // gemm_nt's small-grid split over K: 0 = its own choice, else forced (sweeps)
}

#define SL_CHECK_LAUNCH() (hipGetLastError())
