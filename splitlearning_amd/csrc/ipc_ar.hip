// One-kernel all-reduce over peer-mapped HBM for Bob's tensor-parallel step (see ipc_ar.h for
// the protocol and its memory ordering).
//
// The receive regions and flags are allocated uncached (a peer's stores land in this GPU's
// HBM, no L2 line can go stale between parity reuses whatever cache type a mapping gets);
// payload moves as 16-B system-scope write-through stores and cache-bypassing loads; every
// flag is raised behind a system-scope release and every wait ends in an acquire.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "ipc_ar.h"

namespace sl {
namespace {

#define SL_HIP_THROW(cmd)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (cmd);                                                                   \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#cmd ": ") + hipGetErrorString(e_)); \
  } while (0)

// Workgroup c owns floats [c * kIpcChunk, (c + 1) * kIpcChunk) of the message; flag word c.
__global__ __launch_bounds__(kIpcThreads) void ipc_allreduce_kernel(IpcStep s, float* __restrict__ x, int64_t n) {
  const int c = blockIdx.x;
  const int64_t off = (int64_t)c * kIpcChunk + threadIdx.x * 4;
  const bool live = off < n;   // n % 4 == 0 (checked by the launcher)
  float4 v = {0.f, 0.f, 0.f, 0.f};
  if (live) v = *reinterpret_cast<const float4*>(x + off);
  // push: this chunk into slot [par][me] of every rank's region (this rank's own included)
  const int64_t slot = ((int64_t)s.par * s.T + s.me) * s.cap + off;
  if (live)
    for (int r = 0; r < s.T; ++r) ipc_st4(ipc_rsrc(s.P.data[r]), slot, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int64_t fme = ((int64_t)s.par * s.T + s.me) * s.nflags + c;
  __shared__ int s_ok;
  if (threadIdx.x < 64) {
    if (threadIdx.x < s.T) ipc_raise_flag(s.P.flags[threadIdx.x] + fme, s.gen, s.fences);
    // wait for every rank's chunk c of this generation (lane r polls source r)
    const bool ok = ipc_wait_flags(s, threadIdx.x, c);
    if (threadIdx.x == 0) s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  // a wait gave up (dead / stalled peer): leave x as it was, write nothing derived from
  // stale slots (the job aborts on the error word)
  if (!s_ok || !live) return;
  // every slot's load in flight at once, then the fixed-order sum over ranks 0..T-1
  // (bitwise identical on every rank)
  const __amdgpu_buffer_rsrc_t rs = ipc_rsrc(s.P.data[s.me]);
  const int64_t base = (int64_t)s.par * s.T * s.cap + off;
  float4 u[kIpcMaxRanks];
#pragma unroll
  for (int r = 0; r < kIpcMaxRanks; ++r)
    if (r < s.T) u[r] = ipc_ld4(rs, base + (int64_t)r * s.cap);
  float4 acc = u[0];
#pragma unroll
  for (int r = 1; r < kIpcMaxRanks; ++r) {
    if (r < s.T) {
      acc.x += u[r].x;
      acc.y += u[r].y;
      acc.z += u[r].z;
      acc.w += u[r].w;
    }
  }
  *reinterpret_cast<float4*>(x + off) = acc;
}

}  // namespace

hipError_t ipc_allreduce_launch(const IpcStep& s, float* x, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n > s.cap || n % 4 != 0 || (reinterpret_cast<uintptr_t>(x) & 15) != 0 || s.T < 1 || s.T > kIpcMaxRanks ||
      s.me < 0 || s.me >= s.T)
    return hipErrorInvalidValue;
  const int chunks = (int)((n + kIpcChunk - 1) / kIpcChunk);
  if (chunks > s.nflags) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(chunks), dim3(kIpcThreads), 0, st, s, x, n);
  return hipGetLastError();
}

IpcAllReduce::IpcAllReduce(int nranks, int rank, int64_t cap) : nranks_(nranks), rank_(rank) {
  if (nranks < 1 || nranks > kIpcMaxRanks || rank < 0 || rank >= nranks)
    throw std::runtime_error("IpcAllReduce: 1..8 ranks");
  if (cap < 1) throw std::runtime_error("IpcAllReduce: capacity");
  cap_ = (cap + kIpcChunk - 1) / kIpcChunk * kIpcChunk;
  max_chunks_ = std::max((int)(cap_ / kIpcChunk), kIpcFlags);
  const size_t dbytes = sizeof(float) * 2 * (size_t)nranks * (size_t)cap_;
  const size_t fbytes = sizeof(uint32_t) * 2 * (size_t)nranks * (size_t)max_chunks_;
  if (dbytes / 4 > 0x7fffffff / 4) throw std::runtime_error("IpcAllReduce: region above 2 GB");
  SL_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&data_), dbytes, hipDeviceMallocUncached));
  SL_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), fbytes, hipDeviceMallocUncached));
  SL_HIP_THROW(hipMemset(flags_, 0, fbytes));
  SL_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&err_), sizeof(int), hipDeviceMallocUncached));
  SL_HIP_THROW(hipMemset(err_, 0, sizeof(int)));
  SL_HIP_THROW(hipHostMalloc(reinterpret_cast<void**>(&herr_), sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *herr_ = 0;
  SL_HIP_THROW(hipHostGetDevicePointer(reinterpret_cast<void**>(&herr_dev_), herr_, 0));
  SL_HIP_THROW(hipDeviceSynchronize());
  int dev = 0, khz = 0;
  SL_HIP_THROW(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  clock_khz_ = khz;
  set_timeout_s(30.0);
}

IpcAllReduce::~IpcAllReduce() {
  for (void* p : mapped_) hipIpcCloseMemHandle(p);
  if (data_) hipFree(data_);
  if (flags_) hipFree(flags_);
  if (err_) hipFree(err_);
  if (herr_) hipHostFree(herr_);
}

std::string IpcAllReduce::handle() const {
  hipIpcMemHandle_t hd, hf;
  SL_HIP_THROW(hipIpcGetMemHandle(&hd, data_));
  SL_HIP_THROW(hipIpcGetMemHandle(&hf, flags_));
  std::string s(2 * sizeof(hipIpcMemHandle_t), '\0');
  std::memcpy(&s[0], &hd, sizeof(hd));
  std::memcpy(&s[sizeof(hd)], &hf, sizeof(hf));
  return s;
}

void IpcAllReduce::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != nranks_) throw std::runtime_error("IpcAllReduce.open: one handle per rank");
  if (opened_) throw std::runtime_error("IpcAllReduce.open: already open");
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_) {
      peers_.data[r] = data_;
      peers_.flags[r] = flags_;
      continue;
    }
    if (handles[r].size() != 2 * sizeof(hipIpcMemHandle_t)) throw std::runtime_error("IpcAllReduce.open: bad handle");
    hipIpcMemHandle_t hd, hf;
    std::memcpy(&hd, handles[r].data(), sizeof(hd));
    std::memcpy(&hf, handles[r].data() + sizeof(hd), sizeof(hf));
    void* pd = nullptr;
    void* pf = nullptr;
    SL_HIP_THROW(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess));
    mapped_.push_back(pd);
    SL_HIP_THROW(hipIpcOpenMemHandle(&pf, hf, hipIpcMemLazyEnablePeerAccess));
    mapped_.push_back(pf);
    peers_.data[r] = static_cast<float*>(pd);
    peers_.flags[r] = static_cast<uint32_t*>(pf);
  }
  opened_ = true;
}

void IpcAllReduce::allreduce_sum_f32(float* p, size_t n, hipStream_t st) {
  if (!opened_) throw std::runtime_error("IpcAllReduce: open() first");
  if (n % 4 != 0 || (reinterpret_cast<uintptr_t>(p) & 15) != 0)
    throw std::runtime_error("IpcAllReduce: n % 4 != 0 or a buffer not 16-B aligned");
  // a message above the capacity goes as consecutive cap-sized pieces (every rank issues
  // the same sequence, so the generations stay in step)
  for (size_t o = 0; o < n; o += (size_t)cap_) {
    const int64_t m = std::min<int64_t>(cap_, (int64_t)(n - o));
    const IpcStep s = begin_step();
    SL_HIP_THROW(ipc_allreduce_launch(s, p + o, m, st));
  }
}

IpcStep IpcAllReduce::begin_steps(int64_t S) {
  IpcStep s = begin_step();
  if (S > 1) gen_ += (uint32_t)(S - 1);
  return s;
}

IpcStep IpcAllReduce::begin_step() {
  if (!opened_) throw std::runtime_error("IpcAllReduce: open() first");
  ++gen_;
  IpcStep s;
  s.P = peers_;
  s.T = nranks_;
  s.me = rank_;
  s.par = (int)(gen_ & 1u);
  s.gen = gen_;
  s.cap = cap_;
  s.nflags = max_chunks_;
  s.err = err_;
  s.herr = herr_dev_;
  s.timeout = timeout_;
  s.fences = fences_ ? 1 : 0;
  return s;
}

void IpcAllReduce::rearm(uint32_t gen) {
  if ((int32_t)(gen - gen_) < 0) throw std::runtime_error("IpcAllReduce.rearm: generation behind this rank's");
  SL_HIP_THROW(hipDeviceSynchronize());
  SL_HIP_THROW(hipMemset(err_, 0, sizeof(int)));
  SL_HIP_THROW(hipDeviceSynchronize());
  __atomic_store_n(herr_, 0, __ATOMIC_RELEASE);
  gen_ = gen;
}

int IpcAllReduce::error() const {
  int e = 0;
  SL_HIP_THROW(hipMemcpy(&e, err_, sizeof(int), hipMemcpyDeviceToHost));
  return e | host_error();
}

}  // namespace sl
