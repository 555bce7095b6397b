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
// closing barrier is needed.
//
// Memory ordering (HIP / AMDGPU memory model, system scope because the peers are other
// devices):
//   producer  payload: 16-B write-through stores at system scope (sc0 sc1) into the peer's
//             uncached region -> every storing wave `s_waitcnt vmcnt(0)` -> (workgroup
//             barrier when several waves stored) -> ONE lane: a system-scope RELEASE fence,
//             `s_waitcnt vmcnt(0)` (inline: the compiler may drop its own wait after the
//             write-back, MI355X_MICROARCH.md "Compiler hazard") -> relaxed flag store;
//   consumer  relaxed polls of its own flag words (no acquire per poll: 2-3x slower per hop)
//             -> ONE system-scope ACQUIRE fence once the flag matched -> workgroup barrier
//             -> the slot reads (system-scope sc0 sc1 loads).
// Failure: every wait is bounded (wall clock); a timeout raises the error word, and every
// later wait (this kernel or any later step) that finds its flag missing sees the word and
// gives up at once instead of waiting out the timeout again — so a dead peer costs one
// timeout, not one per step.  The word is mirrored into host-pinned memory, which the native
// executor reads every few steps without a device sync (engine.cpp ServerEpoch::run) and
// raises on.
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
  int* err;           // device error word (uncached)
  int* herr;          // host-pinned mirror of it (read by the host without a sync)
  int64_t timeout;    // wall-clock ticks
  int fences;         // 1: release / acquire fences around the flags (default); 0: the
                      // measured-cost A/B only (set_fences(False), scripts/native_ab.py)
};

__device__ __forceinline__ uint32_t ipc_poll_flag(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Release, then the flag: the payload this lane's workgroup stored (drained and barriered by
// the caller) is visible to any agent that observes the flag and acquires.
__device__ __forceinline__ void ipc_raise_flag(uint32_t* f, uint32_t v, int fence = 1) {
  if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void ipc_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

// 16-B payload access at system scope through a buffer resource over a (wave-uniform) region
// base: one write-through store / cache-bypassing load per float4 (sc0 sc1 = cache policy 17).
typedef int ipc_i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ipc_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ void ipc_st4(__amdgpu_buffer_rsrc_t rs, int64_t off_floats, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ipc_i32x4, v), rs, (int)(off_floats * 4), 0, 17);
}

__device__ __forceinline__ float4 ipc_ld4(__amdgpu_buffer_rsrc_t rs, int64_t off_floats) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off_floats * 4), 0, 17));
}

__device__ __forceinline__ bool ipc_failed(const IpcStep& s) {
  return __hip_atomic_load(s.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

__device__ __forceinline__ void ipc_fail(int* err, int* herr) {
  __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (herr) __hip_atomic_store(herr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lanes 0..T-1 of the calling wave each wait for source rank `lane`'s flag word `idx` of this
// generation, then acquire.  Bounded: a missing flag with the error word already set (an
// earlier timeout on this rank) gives up at once; otherwise the wall-clock timeout raises the
// word.  Returns false (uniformly over the wave) when any wait gave up.
__device__ __forceinline__ bool ipc_wait_flags(const IpcStep& s, int lane, int idx) {
  bool ok = true;
  if (lane < s.T) {
    const uint32_t* f = s.P.flags[s.me] + ((int64_t)s.par * s.T + lane) * s.nflags + idx;
    if ((int32_t)(ipc_poll_flag(f) - s.gen) < 0) {
      const uint64_t t0 = wall_clock64();
      while ((int32_t)(ipc_poll_flag(f) - s.gen) < 0) {
        if (ipc_failed(s)) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if ((int64_t)(wall_clock64() - t0) > s.timeout) {
          ipc_fail(s.err, s.herr);
          ok = false;
          break;
        }
      }
    }
  }
  ok = __all(ok);
  if (s.fences) ipc_acquire();
  return ok;
}

hipError_t ipc_allreduce_launch(const IpcStep& s, float* x, int64_t n, hipStream_t st);

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
  // whether a buffer can go through the peer-mapped kernel: n % 4 == 0, n <= cap and a
  // 16-B aligned address (float4 accesses); otherwise the caller uses RCCL
  bool serves(const float* p, size_t n) const {
    return (int64_t)n <= cap_ && n % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  }
  // in-place sum of n floats (n % 4 == 0, 16-B aligned; above cap: cap-sized pieces) over
  // the ranks, on stream st (stream-ordered; NOT capturable: the flag generation is a launch
  // argument, TpComm uses RCCL under capture)
  void allreduce_sum_f32(float* p, size_t n, hipStream_t st);
  // the next generation for a fused consumer (same sequence as allreduce_sum_f32's calls)
  IpcStep begin_step();
  // S consecutive generations for a persistent consumer (csrc/resident.hip: step i of the
  // launch uses gen + i, parity (gen + i) & 1); every rank reserves the same S
  IpcStep begin_steps(int64_t S);
  int flag_words() const { return max_chunks_; }
  int64_t cap() const { return cap_; }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool opened() const { return opened_; }
  // error word: nonzero after a wait timed out.  error() synchronises; host_error() reads
  // the host-pinned mirror without any device call (may lag the device by the work queued)
  int error() const;
  int host_error() const { return __atomic_load_n(herr_, __ATOMIC_ACQUIRE); }
  // bound on every flag wait (default 30 s: far above any host skew between ranks)
  void set_timeout_s(double s) { timeout_ = (int64_t)(s * 1000.0 * clock_khz_); }
  double timeout_s() const { return (double)timeout_ / (1000.0 * clock_khz_); }
  void set_fences(bool on) { fences_ = on; }
  // Re-arm after a failed wait, as one collective step of every rank: the caller has
  // synchronised its device (no kernel of this rank still reads or writes the region) and the
  // ranks have agreed `gen` = the largest generation any of them reserved (generation()).
  // Clears the error word and its host mirror and continues at gen + 1 on every rank: every
  // flag and tagged granule already in the regions carries a generation <= gen, so none can
  // satisfy a later wait, and the parities of the two buffers stay in step across ranks.
  void rearm(uint32_t gen);
  uint32_t generation() const { return gen_; }

 private:
  int nranks_, rank_;
  int64_t cap_;
  int max_chunks_;
  float* data_ = nullptr;
  uint32_t* flags_ = nullptr;
  int* err_ = nullptr;
  int* herr_ = nullptr;        // host-pinned (mapped) mirror of err_
  int* herr_dev_ = nullptr;    // its device address
  IpcPeers peers_{};
  std::vector<void*> mapped_;
  uint32_t gen_ = 0;
  bool opened_ = false;
  int64_t timeout_ = 0;
  int clock_khz_ = 100000;
  bool fences_ = true;
};

}  // namespace sl
