// Bob's tensor-parallel all-reduce over peer-mapped HBM (`_C.IpcAllReduce`).
//
// The row-parallel fc2 of Bob's TP step needs one in-place sum of a 16 x 1000 fp32 partial
// (64 KB) per optimizer step, a latency-bound message: RCCL's ring / tree all-reduce costs
// several dependent link hops per call.  Here every rank exports a small receive region
// (hipIpcGetMemHandle over uncached device memory) and maps every peer's region once;
// the all-reduce is then ONE kernel per step: each workgroup pushes its chunk of the
// partial into slot [me] of every rank's region over the xGMI links (all peers at once,
// one hop), raises a per-chunk flag on every rank, waits for the T flags of its chunk and
// sums the T slots in rank order 0..T-1 — so every rank computes bitwise the same sum, which
// keeps the replicated fc3 and the fc2 epilogue identical across ranks.  Regions are
// double-buffered by step parity and flags carry a monotonic generation, so no reset or
// closing barrier is needed.  Waits are bounded (a timeout raises the error word).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace sl {

constexpr int kIpcMaxRanks = 8;
constexpr int kIpcThreads = 256;
constexpr int kIpcChunk = kIpcThreads * 4;   // floats per workgroup (one float4 per thread)

struct IpcPeers {
  float* data[kIpcMaxRanks];       // rank r's receive region [2][T][cap] floats
  uint32_t* flags[kIpcMaxRanks];   // rank r's flags [2][T][max_chunks]
};

// Flag words per (parity, source) beyond the all-reduce's chunks: the fused server head
// (fused.hip head_fwd_kernel<.., true>) raises one per (row, column slice) workgroup.
constexpr int kIpcFlags = 1024;

// One generation of the protocol handed to a kernel that does the push / wait itself (the
// server head fuses the fc2 all-reduce into its slab reduction, csrc/fused.hip).
struct IpcStep {
  IpcPeers P;
  int T, me, par;
  uint32_t gen;
  int64_t cap;        // floats per slot
  int nflags;         // flag words per (parity, source)
  int* err;
  int64_t timeout;    // wall-clock ticks
};

__device__ __forceinline__ uint32_t ipc_poll_flag(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void ipc_raise_flag(uint32_t* f, uint32_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Payload moves at system scope (each dword a relaxed system-scope atomic: global_store /
// global_load with sc0 sc1), so the protocol follows the memory model whatever cache type
// the driver gives a peer's mapping: a store leaves no dirty line in this GPU's L2 and is
// complete at `s_waitcnt vmcnt(0)`; a load never hits a stale line of an earlier generation.
__device__ __forceinline__ void ipc_st4(float* p, float4 v) {
  uint32_t* q = reinterpret_cast<uint32_t*>(p);
  __hip_atomic_store(q + 0, __float_as_uint(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(q + 1, __float_as_uint(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(q + 2, __float_as_uint(v.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(q + 3, __float_as_uint(v.w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ float4 ipc_ld4(const float* p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
  float4 v;
  v.x = __uint_as_float(__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  v.y = __uint_as_float(__hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  v.z = __uint_as_float(__hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  v.w = __uint_as_float(__hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  return v;
}

// Lanes 0..T-1 of the calling wave each wait for source rank `lane`'s flag word `idx` of this
// generation (bounded: a timeout raises *err and gives up).
__device__ __forceinline__ void ipc_wait_flags(const IpcStep& s, int lane, int idx) {
  if (lane < s.T) {
    const uint32_t* f = s.P.flags[s.me] + ((int64_t)s.par * s.T + lane) * s.nflags + idx;
    const uint64_t t0 = wall_clock64();
    while ((int32_t)(ipc_poll_flag(f) - s.gen) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if ((int64_t)(wall_clock64() - t0) > s.timeout) {
        atomicOr(s.err, 1);
        break;
      }
    }
  }
}

hipError_t ipc_allreduce_launch(const IpcPeers& P, float* x, int64_t n, int T, int me, uint32_t gen, int64_t cap,
                                int max_chunks, int* err, int64_t timeout_ticks, hipStream_t st);

class IpcAllReduce {
 public:
  // cap: the largest all-reduce (floats) this object serves
  IpcAllReduce(int nranks, int rank, int64_t cap);
  ~IpcAllReduce();
  IpcAllReduce(const IpcAllReduce&) = delete;
  IpcAllReduce& operator=(const IpcAllReduce&) = delete;
  // this rank's two IPC handles (data region, flag region), concatenated
  std::string handle() const;
  // every rank's handle() in rank order; maps the peers' regions
  void open(const std::vector<std::string>& handles);
  // in-place sum of n floats (n % 4 == 0; above cap: cap-sized pieces) over the ranks, on stream st (stream-ordered; NOT
  // capturable: the flag generation is a launch argument, TpComm uses RCCL under capture)
  void allreduce_sum_f32(float* p, size_t n, hipStream_t st);
  // the next generation for a fused consumer (same sequence as allreduce_sum_f32's calls)
  IpcStep begin_step();
  int64_t cap() const { return cap_; }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool opened() const { return opened_; }
  // device error word: nonzero after a wait timed out (synchronising read)
  int error() const;
  // bound on every flag wait (default 30 s: far above any host skew between ranks)
  void set_timeout_s(double s) { timeout_ = (int64_t)(s * 1000.0 * clock_khz_); }

 private:
  int nranks_, rank_;
  int64_t cap_;
  int max_chunks_;
  float* data_ = nullptr;
  uint32_t* flags_ = nullptr;
  int* err_ = nullptr;
  IpcPeers peers_{};
  std::vector<void*> mapped_;
  uint32_t gen_ = 0;
  bool opened_ = false;
  int64_t timeout_ = 0;
  int clock_khz_ = 100000;
};

}  // namespace sl
