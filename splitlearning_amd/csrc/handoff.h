// Hand-off stress test of the persistent kernels' publication primitive (csrc/handoff.hip).
#pragma once
#include <string>

#include "common.h"

namespace sl {

constexpr int kHoThreads = 512;
constexpr int kHoStride = 32;          // counter shards 128 B apart
constexpr int kHoScratchF4 = 4096;     // float4 of scratch per workgroup (64 KB)

struct HoArgs {
  float* D;            // [G][P] payload, rewritten in place every round
  float* scratch;      // [G][kHoScratchF4] float4: the bandwidth stream of the uneven load
  unsigned* cnt;       // [2 seams][8 shards][kHoStride] arrival counters (zeroed per launch)
  unsigned* bad;       // [G] mismatching words seen by each consumer
  unsigned* done;      // [G] last round each workgroup completed
  unsigned* first;     // [8] {count, round, src, idx, got, want, consumer} of the first mismatch
  int* err;            // nonzero after a wait gave up
  int64_t timeout;     // wall-clock ticks per wait
  int P, R, nsrc, src_stride, mode;
  int busy_ticks;      // random per-round delay bound (wall-clock ticks; 0 = none)
};

std::string handoff_check(const HoArgs& a, int G);
hipError_t handoff_stress_launch(const HoArgs& a, int G, hipStream_t st);

}  // namespace sl
