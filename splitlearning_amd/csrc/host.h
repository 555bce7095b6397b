// Host-side helpers shared by the bindings and the native executors: optimizer and
// epilogue descriptors, and the per-(layer, step) dropout seed (bit-identical to
// ops/rng.py::step_seed).
#pragma once
#include <cmath>
#include <cstdint>

#include "common.h"

namespace sl {

// kind 0 = gradient only, 1 = SGD(momentum), 2 = Adam (L2 wd).  Adam's bias corrections for
// step t (>= 1) are folded into {step_size, inv_bc2_sqrt} unless `dyn` supplies them.
inline SlOpt make_opt_raw(int kind, double lr, double beta1, double beta2, double eps, double wd, double momentum,
                          int64_t t, const float* dyn) {
  SlOpt o{};
  o.kind = kind;
  o.lr = (float)lr;
  o.beta1 = (float)beta1;
  o.beta2 = (float)beta2;
  o.eps = (float)eps;
  o.wd = (float)wd;
  o.momentum = (float)momentum;
  o.dyn = dyn;
  if (kind == 2 && !dyn && t >= 1) {
    const double bc1 = 1.0 - std::pow(beta1, (double)t);
    const double bc2 = 1.0 - std::pow(beta2, (double)t);
    o.step_size = (float)(lr / bc1);
    o.inv_bc2_sqrt = (float)(1.0 / std::sqrt(bc2));
  }
  return o;
}

inline Epi make_epi_raw(const float* bias, bool relu, double drop_p, uint64_t seed, int col_off,
                        const uint32_t* dseed) {
  Epi e{};
  e.bias = bias;
  e.relu = relu ? 1 : 0;
  e.thresh = drop_p > 0 ? (uint32_t)(drop_p * 4294967296.0) : 0u;
  e.dscale = drop_p > 0 ? (float)(1.0 / (1.0 - drop_p)) : 1.f;
  e.seed_lo = (uint32_t)(seed & 0xffffffffull);
  e.seed_hi = (uint32_t)(seed >> 32);
  e.col_off = col_off;
  e.dseed = dseed;
  return e;
}

inline uint64_t step_seed(uint64_t base, uint64_t layer, uint64_t step) {
  uint64_t x = base * 0x9E3779B97F4A7C15ull + layer * 0xBF58476D1CE4E5B9ull + step * 0x94D049BB133111EBull;
  x ^= x >> 31;
  x *= 0xD6E8FEB86659FD93ull;
  x ^= x >> 32;
  return x;
}

}  // namespace sl
