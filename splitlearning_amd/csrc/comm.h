// Native RCCL communicator shared by the Python bindings (comm.cpp) and the native
// server-epoch executor (engine.cpp), which issues Bob's per-step all-reduce itself.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <string>

#include "ipc_ar.h"

namespace sl {

class TpComm {
 public:
  TpComm(const std::string& uid, int nranks, int rank);
  ~TpComm();
  TpComm(const TpComm&) = delete;
  TpComm& operator=(const TpComm&) = delete;
  // in-place sum of n floats on stream st (the data plane of Bob's TP step): the attached
  // peer-mapped all-reduce (ipc_ar.h) when one is attached, n fits (n <= cap, n % 4 == 0)
  // and the stream is not being captured; ncclAllReduce otherwise (capturable)
  void allreduce_sum_f32(float* p, size_t n, hipStream_t st);
  void attach_ipc(IpcAllReduce* a) { ipc_ = a; }
  IpcAllReduce* ipc() const { return ipc_; }
  ncclComm_t get() const { return comm_; }
  int rank() const { return rank_; }
  int size() const { return nranks_; }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
  IpcAllReduce* ipc_ = nullptr;
};

}  // namespace sl
