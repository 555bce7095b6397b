// The fused U-shape middle + head launch (csrc/ushape.hip): arguments and entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.h"

namespace sl {

struct MidArgs {
  const float* pn;      // look-ahead slabs [S][M][N1] (slab stride `slab`), or null: h1 given
  int S;
  int64_t slab;
  Epi e1;               // fc1 epilogue (b1, ReLU)
  float* h1;            // [M][N1]: written when pn, read otherwise
  const float* W2;      // [N2][N1]
  Epi e2;               // fc2 epilogue (b2, ReLU)
  float* h2;            // [M][N2] out
  float* hw;            // head W [C][N2] (updated in place)
  float* hb;            // head b [C]
  float *s0w, *s1w, *s0b, *s1b;
  const int64_t* y;
  int64_t ignore;
  float scale;
  float* loss_rows;     // [M]
  float* dz2;           // [M][N2] out: dL/dh2 masked by [h2 > 0]
  SlOpt o;              // the head's optimizer step
  float* part;          // [J][ceil(N2 / 16)][64] f32x4 partials
  unsigned* cnt;        // arrival counter, 0 between launches
  int M, N1, N2, C;
};

// Whether the fused launch covers this shape (fp32, M <= 16, N1 <= 1024, N2 <= 128, C <= 16).
bool ushape_mid_ok(int M, int N1, int N2, int C);
// Its partial workspace in floats.
int64_t ushape_mid_part_floats(int N1, int N2);
hipError_t ushape_mid(const MidArgs& a, hipStream_t st);

}  // namespace sl
