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

#include "comm.h"
#include "ipc_p2p.h"

namespace py = pybind11;

#define SL_NCCL(cmd)                                                                        \
  do {                                                                                      \
    ncclResult_t r_ = (cmd);                                                                \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error '", ncclGetErrorString(r_), "' in " #cmd); \
  } while (0)

namespace sl {

TpComm::TpComm(const std::string& uid, int nranks, int rank) : nranks_(nranks), rank_(rank) {
  TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "bad RCCL unique id size");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  SL_NCCL(ncclCommInitRank(&comm_, nranks, id, rank));
}

TpComm::~TpComm() {
  if (comm_) ncclCommDestroy(comm_);
}

void TpComm::allreduce_sum_f32(float* p, size_t n, hipStream_t st) {
  if (ipc_ != nullptr && ipc_->serves(p, n)) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    // a captured launch would freeze the flag generation into the graph: RCCL there
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
      ipc_->allreduce_sum_f32(p, n, st);
      return;
    }
  }
  SL_NCCL(ncclAllReduce(p, p, n, ncclFloat32, ncclSum, comm_, st));
}

}  // namespace sl

namespace {

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

// Python-facing methods on tensors (the class itself is sl::TpComm, comm.h)
void allreduce_sum(sl::TpComm& c, at::Tensor& t) {
  need(t);
  if (t.scalar_type() == at::kFloat) {
    c.allreduce_sum_f32(t.data_ptr<float>(), (size_t)t.numel(), stream());
    return;
  }
  SL_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), ncclSum, c.get(), stream()));
}
void broadcast(sl::TpComm& c, at::Tensor& t, int root) {
  need(t);
  SL_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), root, c.get(), stream()));
}
void all_gather(sl::TpComm& c, at::Tensor& out, const at::Tensor& in) {
  need(out);
  need(in);
  TORCH_CHECK(out.numel() == in.numel() * c.size() && out.scalar_type() == in.scalar_type(), "all_gather sizes");
  SL_NCCL(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), dtype_of(in), c.get(), stream()));
}
void send(sl::TpComm& c, const at::Tensor& t, int peer) {
  need(t);
  SL_NCCL(ncclSend(t.data_ptr(), t.numel(), dtype_of(t), peer, c.get(), stream()));
}
void recv(sl::TpComm& c, at::Tensor& t, int peer) {
  need(t);
  SL_NCCL(ncclRecv(t.data_ptr(), t.numel(), dtype_of(t), peer, c.get(), stream()));
}

py::bytes unique_id() {
  ncclUniqueId id;
  SL_NCCL(ncclGetUniqueId(&id));
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

}  // namespace

void sl_register_comm(py::module& m) {
  py::class_<sl::TpComm>(m, "TpComm")
      .def(py::init([](const py::bytes& uid, int nranks, int rank) {
        return new sl::TpComm(std::string(uid), nranks, rank);
      }))
      .def("allreduce_sum", &allreduce_sum)
      .def("broadcast", &broadcast)
      .def("all_gather", &all_gather)
      .def("send", &send)
      .def("recv", &recv)
      .def("group_start", [](sl::TpComm&) { SL_NCCL(ncclGroupStart()); })
      .def("group_end", [](sl::TpComm&) { SL_NCCL(ncclGroupEnd()); })
      .def("attach_ipc", [](sl::TpComm& c, sl::IpcAllReduce* a) { c.attach_ipc(a); }, py::keep_alive<1, 2>(),
           py::arg("ipc").none(true))
      .def_property_readonly("ipc_attached", [](const sl::TpComm& c) { return c.ipc() != nullptr; })
      .def_property_readonly("rank", &sl::TpComm::rank)
      .def_property_readonly("size", &sl::TpComm::size);
  py::class_<sl::IpcAllReduce>(m, "IpcAllReduce")
      .def(py::init<int, int, int64_t>(), py::arg("nranks"), py::arg("rank"), py::arg("cap"))
      .def("handle", [](const sl::IpcAllReduce& a) { return py::bytes(a.handle()); })
      .def("open", [](sl::IpcAllReduce& a, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (const auto& h : hs) v.emplace_back(std::string(h));
        a.open(v);
      })
      .def("allreduce_sum", [](sl::IpcAllReduce& a, at::Tensor& t) {
        need(t);
        TORCH_CHECK(t.scalar_type() == at::kFloat, "IpcAllReduce: f32");
        a.allreduce_sum_f32(t.data_ptr<float>(), (size_t)t.numel(), stream());
      })
      .def("error", &sl::IpcAllReduce::error)
      .def("host_error", &sl::IpcAllReduce::host_error)
      .def("set_fences", &sl::IpcAllReduce::set_fences)
      .def("set_timeout_s", &sl::IpcAllReduce::set_timeout_s)
      .def("rearm", &sl::IpcAllReduce::rearm, py::arg("gen"))
      .def_property_readonly("generation", &sl::IpcAllReduce::generation)
      .def_property_readonly("timeout_s", &sl::IpcAllReduce::timeout_s)
      .def_property_readonly("cap", &sl::IpcAllReduce::cap)
      .def_property_readonly("rank", &sl::IpcAllReduce::rank)
      .def_property_readonly("size", &sl::IpcAllReduce::size);
  py::class_<sl::IpcChannel>(m, "IpcChannel")
      .def(py::init<int, int, int64_t>(), py::arg("nranks"), py::arg("rank"), py::arg("cap"))
      .def("handle", [](const sl::IpcChannel& a) { return py::bytes(a.handle()); })
      .def("open", [](sl::IpcChannel& a, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (const auto& h : hs) v.emplace_back(std::string(h));
        a.open(v);
      })
      // tensor-level send / recv (any dtype, viewed as 4-byte words) on the current stream
      .def("send", [](sl::IpcChannel& a, const at::Tensor& t, int peer) {
        need(t);
        TORCH_CHECK(t.nbytes() % 16 == 0, "IpcChannel: messages are whole 16-byte units");
        a.send(static_cast<const float*>(t.data_ptr()), (int64_t)(t.nbytes() / 4), peer, stream());
      })
      .def("recv", [](sl::IpcChannel& a, at::Tensor& t, int peer) {
        need(t);
        TORCH_CHECK(t.nbytes() % 16 == 0, "IpcChannel: messages are whole 16-byte units");
        a.recv(static_cast<float*>(t.data_ptr()), (int64_t)(t.nbytes() / 4), peer, stream());
      })
      .def("error", &sl::IpcChannel::error)
      .def("host_error", &sl::IpcChannel::host_error)
      .def("set_timeout_s", &sl::IpcChannel::set_timeout_s)
      .def("sent", &sl::IpcChannel::sent)
      .def("received", &sl::IpcChannel::received)
      .def_property_readonly("timeout_s", &sl::IpcChannel::timeout_s)
      .def_property_readonly("cap", &sl::IpcChannel::cap)
      .def_property_readonly("rank", &sl::IpcChannel::rank)
      .def_property_readonly("size", &sl::IpcChannel::size);
  m.def("nccl_unique_id", &unique_id);
  int v = 0;
  ncclGetVersion(&v);
  m.attr("rccl_version") = v;
}
