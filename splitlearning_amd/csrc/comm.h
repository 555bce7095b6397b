// Native RCCL communicator shared by the Python bindings (comm.cpp) and the native
// server-epoch executor (engine.cpp), which issues Bob's per-step all-reduce itself.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <string>

namespace sl {

class TpComm {
 public:
  TpComm(const std::string& uid, int nranks, int rank);
  ~TpComm();
  TpComm(const TpComm&) = delete;
  TpComm& operator=(const TpComm&) = delete;
  // in-place sum of n floats on stream st (capturable; the data plane of Bob's TP step)
  void allreduce_sum_f32(float* p, size_t n, hipStream_t st);
  ncclComm_t get() const { return comm_; }
  int rank() const { return rank_; }
  int size() const { return nranks_; }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
};

}  // namespace sl
