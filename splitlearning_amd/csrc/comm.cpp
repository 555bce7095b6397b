// Native RCCL communicator for the data plane (tensor-parallel Bob and p2p transfers).
//
// Why not only torch.distributed: the per-step all-reduce of Bob's tensor-parallel
// fc2 partial sums sits in the middle of the server step, and the step is replayed as a
// HIP graph.  ncclAllReduce issued on the caller's stream from C++ is capturable and has
// no Python / ProcessGroup bookkeeping on the hot path.  The communicator is created from
// a unique id that Python broadcasts over the existing torch.distributed group (so
// rendezvous, timeouts and failure detection stay with the control plane).  It links the
// same librccl.so.1 that PyTorch-ROCm loads (one RCCL instance per process).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

namespace py = pybind11;

namespace {

#define SL_NCCL(cmd)                                                                        \
  do {                                                                                      \
    ncclResult_t r_ = (cmd);                                                                \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error '", ncclGetErrorString(r_), "' in " #cmd); \
  } while (0)

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
}

void need(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL tensors must be contiguous GPU tensors");
}

class TpComm {
 public:
  TpComm(const py::bytes& uid, int nranks, int rank) : nranks_(nranks), rank_(rank) {
    std::string s = uid;
    TORCH_CHECK(s.size() == NCCL_UNIQUE_ID_BYTES, "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
    SL_NCCL(ncclCommInitRank(&comm_, nranks, id, rank));
  }
  ~TpComm() {
    if (comm_) ncclCommDestroy(comm_);
  }
  void allreduce_sum(at::Tensor& t) {
    need(t);
    SL_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), ncclSum, comm_, stream()));
  }
  void broadcast(at::Tensor& t, int root) {
    need(t);
    SL_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), root, comm_, stream()));
  }
  void all_gather(at::Tensor& out, const at::Tensor& in) {
    need(out);
    need(in);
    TORCH_CHECK(out.numel() == in.numel() * nranks_ && out.scalar_type() == in.scalar_type(), "all_gather sizes");
    SL_NCCL(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), dtype_of(in), comm_, stream()));
  }
  void send(const at::Tensor& t, int peer) {
    need(t);
    SL_NCCL(ncclSend(t.data_ptr(), t.numel(), dtype_of(t), peer, comm_, stream()));
  }
  void recv(at::Tensor& t, int peer) {
    need(t);
    SL_NCCL(ncclRecv(t.data_ptr(), t.numel(), dtype_of(t), peer, comm_, stream()));
  }
  void group_start() { SL_NCCL(ncclGroupStart()); }
  void group_end() { SL_NCCL(ncclGroupEnd()); }
  int rank() const { return rank_; }
  int size() const { return nranks_; }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
};

py::bytes unique_id() {
  ncclUniqueId id;
  SL_NCCL(ncclGetUniqueId(&id));
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

}  // namespace

void sl_register_comm(py::module& m) {
  py::class_<TpComm>(m, "TpComm")
      .def(py::init<const py::bytes&, int, int>())
      .def("allreduce_sum", &TpComm::allreduce_sum)
      .def("broadcast", &TpComm::broadcast)
      .def("all_gather", &TpComm::all_gather)
      .def("send", &TpComm::send)
      .def("recv", &TpComm::recv)
      .def("group_start", &TpComm::group_start)
      .def("group_end", &TpComm::group_end)
      .def_property_readonly("rank", &TpComm::rank)
      .def_property_readonly("size", &TpComm::size);
  m.def("nccl_unique_id", &unique_id);
  int v = 0;
  ncclGetVersion(&v);
  m.attr("rccl_version") = v;
}
