// Point-to-point messages over peer-mapped HBM (see ipc_p2p.h for the protocol).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "ipc_p2p.h"

namespace sl {
namespace {

#define SL_HIP_THROW(cmd)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (cmd);                                                                   \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#cmd ": ") + hipGetErrorString(e_)); \
  } while (0)

// One lane: wait until *w >= want (generation order), bounded; see ipc_ar.h ipc_wait_flags
__device__ bool p2p_wait(const uint32_t* w, uint32_t want, const P2PMsg& m) {
  if ((int32_t)(ipc_poll_flag(w) - want) >= 0) return true;
  const uint64_t t0 = wall_clock64();
  while ((int32_t)(ipc_poll_flag(w) - want) < 0) {
    if (__hip_atomic_load(m.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return false;
    __builtin_amdgcn_s_sleep(1);
    if ((int64_t)(wall_clock64() - t0) > m.timeout) {
      ipc_fail(m.err, m.herr);
      return false;
    }
  }
  return true;
}

// Workgroup c moves floats [c * kIpcChunk, (c + 1) * kIpcChunk).  prev: chunk count of the
// message two generations back (it used the same parity slot); chunks beyond it were last
// written by a message the receiver had fully read before it acked any chunk of that one
// (its receives of this pair run in stream order), so they wait on chunk 0's ack.
__global__ __launch_bounds__(kIpcThreads) void p2p_send_kernel(P2PMsg m, const float* __restrict__ x, int64_t n,
                                                               int prev) {
  const int c = blockIdx.x;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    bool ok = true;
    if (prev > 0) ok = p2p_wait(m.ack + (c < prev ? c : 0), m.gen - 2, m);
    ipc_acquire();
    s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  if (!s_ok) return;
  const int64_t off = (int64_t)c * kIpcChunk + threadIdx.x * 4;
  if (off < n) ipc_st4(ipc_rsrc(m.data), off, *reinterpret_cast<const float4*>(x + off));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) ipc_raise_flag(m.flag + c, m.gen);
}

__global__ __launch_bounds__(kIpcThreads) void p2p_recv_kernel(P2PMsg m, float* __restrict__ x, int64_t n) {
  const int c = blockIdx.x;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    const bool ok = p2p_wait(m.flag + c, m.gen, m);
    ipc_acquire();
    s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  if (!s_ok) return;   // a wait gave up: nothing derived from a stale slot is written
  const int64_t off = (int64_t)c * kIpcChunk + threadIdx.x * 4;
  if (off < n) *reinterpret_cast<float4*>(x + off) = ipc_ld4(ipc_rsrc(m.data), off);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) ipc_raise_flag(m.ack + c, m.gen);
}

}  // namespace

IpcChannel::IpcChannel(int nranks, int rank, int64_t cap) : nranks_(nranks), rank_(rank) {
  if (nranks < 1 || nranks > kIpcMaxRanks || rank < 0 || rank >= nranks)
    throw std::runtime_error("IpcChannel: 1..8 ranks");
  if (cap < 1) throw std::runtime_error("IpcChannel: capacity");
  cap_ = (cap + kIpcChunk - 1) / kIpcChunk * kIpcChunk;
  nch_ = (int)(cap_ / kIpcChunk);
  const size_t dbytes = sizeof(float) * (size_t)nranks * 2 * (size_t)cap_;
  const size_t sbytes = sizeof(uint32_t) * 2 * (size_t)nranks * 2 * (size_t)nch_;
  if (sizeof(float) * 2 * (size_t)cap_ > 0x7fffffffu) throw std::runtime_error("IpcChannel: slot above 2 GB");
  SL_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&data_), dbytes, hipDeviceMallocUncached));
  SL_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&syncw_), sbytes, hipDeviceMallocUncached));
  SL_HIP_THROW(hipMemset(syncw_, 0, sbytes));
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
  send_gen_.assign(nranks, 0);
  recv_gen_.assign(nranks, 0);
  hist_.assign(2 * nranks, 0);
}

IpcChannel::~IpcChannel() {
  for (void* p : mapped_) hipIpcCloseMemHandle(p);
  if (data_) hipFree(data_);
  if (syncw_) hipFree(syncw_);
  if (err_) hipFree(err_);
  if (herr_) hipHostFree(herr_);
}

std::string IpcChannel::handle() const {
  hipIpcMemHandle_t hd, hs;
  SL_HIP_THROW(hipIpcGetMemHandle(&hd, data_));
  SL_HIP_THROW(hipIpcGetMemHandle(&hs, syncw_));
  std::string s(2 * sizeof(hipIpcMemHandle_t), '\0');
  std::memcpy(&s[0], &hd, sizeof(hd));
  std::memcpy(&s[sizeof(hd)], &hs, sizeof(hs));
  return s;
}

void IpcChannel::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != nranks_) throw std::runtime_error("IpcChannel.open: one handle per rank");
  if (opened_) throw std::runtime_error("IpcChannel.open: already open");
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_) {
      peer_data_[r] = data_;
      sync_[r] = syncw_;
      continue;
    }
    if (handles[r].empty()) continue;   // a rank this one never talks to
    if (handles[r].size() != 2 * sizeof(hipIpcMemHandle_t)) throw std::runtime_error("IpcChannel.open: bad handle");
    hipIpcMemHandle_t hd, hs;
    std::memcpy(&hd, handles[r].data(), sizeof(hd));
    std::memcpy(&hs, handles[r].data() + sizeof(hd), sizeof(hs));
    void* pd = nullptr;
    void* ps = nullptr;
    SL_HIP_THROW(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess));
    mapped_.push_back(pd);
    SL_HIP_THROW(hipIpcOpenMemHandle(&ps, hs, hipIpcMemLazyEnablePeerAccess));
    mapped_.push_back(ps);
    peer_data_[r] = static_cast<float*>(pd);
    sync_[r] = static_cast<uint32_t*>(ps);
  }
  opened_ = true;
}

void IpcChannel::check(const void* x, int64_t n, int peer) const {
  if (!opened_) throw std::runtime_error("IpcChannel: open() first");
  if (peer < 0 || peer >= nranks_ || peer == rank_ || sync_[peer] == nullptr)
    throw std::runtime_error("IpcChannel: peer " + std::to_string(peer) + " not mapped");
  if (!serves(x, n))
    throw std::runtime_error("IpcChannel: message of " + std::to_string(n) +
                             " floats (needs n % 4 == 0, n <= cap, a 16-B aligned buffer)");
}

void IpcChannel::bind_stream(std::vector<hipStream_t>& sts, std::vector<char>& bound, int peer, hipStream_t st,
                             const char* what) {
  if (sts.size() < (size_t)nranks_) {
    sts.assign(nranks_, nullptr);
    bound.assign(nranks_, 0);
  }
  if (!bound[peer]) {
    bound[peer] = 1;
    sts[peer] = st;
  } else if (sts[peer] != st) {
    throw std::runtime_error(std::string("IpcChannel.") + what + ": every message of a pair must be issued on one "
                             "stream (the per-chunk acks are ordered by it)");
  }
}

void IpcChannel::send(const float* x, int64_t n, int peer, hipStream_t st) {
  if (n == 0) return;
  check(x, n, peer);
  bind_stream(send_st_, send_bound_, peer, st, "send");
  const uint32_t g = ++send_gen_[peer];
  const int par = (int)(g & 1u);
  const int chunks = (int)((n + kIpcChunk - 1) / kIpcChunk);
  P2PMsg m{peer_data_[peer] + ((int64_t)rank_ * 2 + par) * cap_, sync_[peer] + flag_off(rank_, par),
           syncw_ + ack_off(peer, par), g, err_, herr_dev_, timeout_};
  int& prev = hist_[2 * peer + par];
  hipLaunchKernelGGL(p2p_send_kernel, dim3(chunks), dim3(kIpcThreads), 0, st, m, x, n, prev);
  SL_HIP_THROW(hipGetLastError());
  prev = chunks;
}

void IpcChannel::recv(float* x, int64_t n, int peer, hipStream_t st) {
  if (n == 0) return;
  check(x, n, peer);
  bind_stream(recv_st_, recv_bound_, peer, st, "recv");
  const uint32_t g = ++recv_gen_[peer];
  const int par = (int)(g & 1u);
  const int chunks = (int)((n + kIpcChunk - 1) / kIpcChunk);
  P2PMsg m{data_ + ((int64_t)peer * 2 + par) * cap_, syncw_ + flag_off(peer, par), sync_[peer] + ack_off(rank_, par),
           g, err_, herr_dev_, timeout_};
  hipLaunchKernelGGL(p2p_recv_kernel, dim3(chunks), dim3(kIpcThreads), 0, st, m, x, n);
  SL_HIP_THROW(hipGetLastError());
}

P2PRun IpcChannel::run(int peer, hipStream_t st, const std::vector<int64_t>& sends,
                       const std::vector<int64_t>& recvs) {
  for (int64_t n : sends) check(data_, n, peer);
  for (int64_t n : recvs) check(data_, n, peer);
  if (!sends.empty()) bind_stream(send_st_, send_bound_, peer, st, "send");
  if (!recvs.empty()) bind_stream(recv_st_, recv_bound_, peer, st, "recv");
  P2PRun r{};
  for (int par = 0; par < 2; ++par) {
    r.sdata[par] = peer_data_[peer] + ((int64_t)rank_ * 2 + par) * cap_;
    r.sflag[par] = sync_[peer] + flag_off(rank_, par);
    r.sack[par] = syncw_ + ack_off(peer, par);
    r.rdata[par] = data_ + ((int64_t)peer * 2 + par) * cap_;
    r.rflag[par] = syncw_ + flag_off(peer, par);
    r.rack[par] = sync_[peer] + ack_off(rank_, par);
  }
  r.sgen0 = send_gen_[peer];
  r.rgen0 = recv_gen_[peer];
  for (int j = 0; j < 2; ++j) r.sprev[j] = hist_[2 * peer + (int)((r.sgen0 + 1u + (uint32_t)j) & 1u)];
  for (int64_t n : sends) {
    const uint32_t g = ++send_gen_[peer];
    hist_[2 * peer + (int)(g & 1u)] = (int)((n + kIpcChunk - 1) / kIpcChunk);
  }
  recv_gen_[peer] += (uint32_t)recvs.size();
  r.err = err_;
  r.herr = herr_dev_;
  r.timeout = timeout_;
  return r;
}

int IpcChannel::error() const {
  int e = 0;
  SL_HIP_THROW(hipMemcpy(&e, err_, sizeof(int), hipMemcpyDeviceToHost));
  return e | host_error();
}

}  // namespace sl
