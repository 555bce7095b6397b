// Native executor of a split-mode epoch (`_C.SplitEpoch`): vanilla and U-shape training of
// one Alice whose Bob is a single shard in the same process (one GPU: the BASELINE ws = 2 point
// and every co-located placement with Bob TP = 1).
//
// Reference hot loops: vanilla data_entities_vanilla.py:66-76 (per batch: Alice forward ->
// bob.train_and_backward over RPC -> dist-autograd backward -> DistributedOptimizer step),
// U-shape data_entities.py:65-81 (Alice front -> bob.inference -> Alice head + CE -> backward
// through Bob to Alice -> one Adam over all three).  The Python epoch (protocols/vanilla.py,
// protocols/ushape.py `split_epoch`, look-ahead order) issues ~10 launches per batch from
// Python; this class issues the SAME launches with the same arguments, seeds, workspace sizes
// and optimizer step counts from C++, so the results are bit-identical
// (tests/test_split_native_gpu.py):
//
//   Alice   conv forward of batch i (gathers its labels; applies her pending update in-kernel)
//   Bob     [fc1 epilogue of the look-ahead slabs | fc1 forward] -> fc2 ...
//     vanilla: fc2 split-K forward, head_fwd + head_bwd (CE on Bob), fc2 dgrad, fc1 dgrad -> dx
//     U-shape: fc2 forward (+ReLU) -> Alice's head step (head + CE + dL/dmid, her head update,
//              Bob's last ReLU mask) -> fc2 dgrad -> fc1 dgrad -> dx
//   Alice   conv backward from dx: dW partials; the pending update of batch i-1 is stored
//   Alice   conv forward of batch i+1 (the update of batch i applied in-kernel)
//   Bob     grouped wgrad + optimizer of every layer, with batch i+1's fc1 product (look-ahead)
//   end     the last pending Alice update is stored
//
// Remote placements (role 1 = the Alice's process, role 2 = Bob's, Bob one shard): each side
// issues ITS half of the same loop, and the per-batch messages go through a link on the
// compute stream -- the peer-mapped channel (csrc/ipc_p2p.h; ranks sharing one GPU, and
// the low-latency path across xGMI) or the RCCL communicator (ncclSend / ncclRecv):
//   vanilla  Alice -> Bob  [act | labels as int64 words]  Bob -> Alice  dx
//   U-shape  Alice -> Bob  act;  Bob -> Alice  mid;  Alice -> Bob  d(mid);  Bob -> Alice  dx
// With the Alice remote there is no look-ahead (VanillaSession.split_epoch's overlap
// order, data_entities_vanilla.py:66-76): Bob's update of batch i is issued right after dx
// leaves, so it runs while she does her backward and next forward; his next fc1 forward
// re-reads fc1.  Same launches, arguments and step counts as the Python loop of that
// placement (tests/test_split_native_gpu.py::test_remote_*).
//
// (Running fc2 / fc3's update on a side stream beside the Alice's backward + next forward, fc1
// alone on the main stream, measured slower: 87-88 k vs 92-94 k samples/s at vanilla ws = 2,
// profiles/r3_vanilla_side_stream_ab.txt.)
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <tuple>
#include <vector>

#include "comm.h"
#include "common.h"
#include "fused.h"
#include "host.h"
#include "ipc_p2p.h"

namespace sl {
hipError_t conv_fwd(const void* x, bool x_u8, const int64_t* idx, int64_t row0, int B, const float* w,
                    const float* b, float* y, uint8_t* am, hipStream_t st, const int64_t* lab_in,
                    int64_t* lab_out, const ConvPending* pend);
hipError_t conv_bwd_step(const float* dy, const float* y, const uint8_t* am, const void* x, bool x_u8,
                         const int64_t* idx, int B, float* w, float* b, float* slab, float* s0w, float* s1w,
                         float* s0b, float* s1b, SlOpt o, hipStream_t st, bool defer, const ConvPending* pend);
hipError_t conv_apply(const ConvPending& p, float* w, float* b, hipStream_t st);
hipError_t head_step(const float* X, float* W, float* b, const int64_t* y, int64_t ignore, float scale,
                     float* loss_rows, float* dX, float* s0w, float* s1w, float* s0b, float* s1b, int M, int K, int C,
                     SlOpt o, bool mask_dx, hipStream_t st);
hipError_t linear_fwd(const float* X, int ldx, const float* W, int ldw, float* Y, int ldy, int M, int N, int K,
                      Epi e, float* ws, int64_t ws_elems, hipStream_t st);
hipError_t linear_dgrad(const float* dZ, int ldz, const float* W, int ldw, const float* hprev, int ldh,
                        float scale, float* dX, int ldx, float* ws, int64_t ws_elems, int M, int N, int K,
                        hipStream_t st);
hipError_t linear_epilogue(const float* P, int ldp, float* Y, int ldy, int M, int N, Epi e, int S, int64_t slab,
                           hipStream_t st);
hipError_t linear_fwd_partial(const float* X, int ldx, const float* W, int ldw, int M, int N, int K, float* ws,
                              int64_t ws_elems, int max_split, int* S_out, hipStream_t st);
}  // namespace sl

namespace py = pybind11;

namespace {

constexpr int kCut = 5408;

void ck(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e)); }

at::Tensor get(const py::dict& d, const char* k) {
  TORCH_CHECK(d.contains(k), "SplitEpoch: missing '", k, "'");
  return d[k].cast<at::Tensor>();
}

float* opt_ptr(const py::dict& d, const char* k) {
  if (!d.contains(k) || d[k].is_none()) return nullptr;
  return d[k].cast<at::Tensor>().data_ptr<float>();
}

void need(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "SplitEpoch: ", what,
              " must be a contiguous f32 GPU tensor");
}

struct Opt {
  int kind = 1;
  double lr = 0, beta1 = 0, beta2 = 0, eps = 0, wd = 0, mom = 0;
  SlOpt at(int64_t t) const { return sl::make_opt_raw(kind, lr, beta1, beta2, eps, wd, mom, t, nullptr); }
};

Opt read_opt(const py::dict& d) {
  Opt o;
  o.kind = d["kind"].cast<int>();
  TORCH_CHECK(o.kind == 1 || o.kind == 2, "SGD-momentum or Adam");
  o.lr = d["lr"].cast<double>();
  o.beta1 = d["beta1"].cast<double>();
  o.beta2 = d["beta2"].cast<double>();
  o.eps = d["eps"].cast<double>();
  o.wd = d["wd"].cast<double>();
  o.mom = d["momentum"].cast<double>();
  return o;
}

// A parameter tensor and its optimizer state (s1 = Adam's v, null for SGD)
struct Param {
  at::Tensor p;
  float* s0 = nullptr;
  float* s1 = nullptr;
};

Param read_param(const py::dict& d, const char* name) {
  const py::dict e = d[name].cast<py::dict>();
  Param q;
  q.p = get(e, "p");
  need(q.p, name);
  q.s0 = opt_ptr(e, "s0");
  q.s1 = opt_ptr(e, "s1");
  TORCH_CHECK(q.s0 != nullptr, "SplitEpoch: ", name, " needs its optimizer state");
  return q;
}

// The vanilla activation message: [M x 5408 activation | M labels as int64 (2 words each)],
// padded to whole 16-byte units (protocols/base.py Session.pack writes the same layout)
int64_t act_msg_words(int M) { return ((int64_t)M * kCut + 2 * (int64_t)M + 3) / 4 * 4; }

// The per-batch message link of a remote placement: the peer-mapped channel or RCCL, on the
// compute stream.  Every message is logged (op, peer, bytes) for the message-sequence tests.
struct Link {
  sl::IpcChannel* ipc = nullptr;
  sl::TpComm* rccl = nullptr;
  int peer = -1;
  std::vector<std::tuple<std::string, int, int64_t>> log;

  void send(const float* p, int64_t n, hipStream_t st) {
    log.emplace_back("send", peer, n * 4);
    if (ipc != nullptr) {
      ipc->send(p, n, peer, st);
      return;
    }
    const ncclResult_t r = ncclSend(p, (size_t)n, ncclFloat32, peer, rccl->get(), st);
    TORCH_CHECK(r == ncclSuccess, "SplitEpoch: ncclSend: ", ncclGetErrorString(r));
  }
  void recv(float* p, int64_t n, hipStream_t st) {
    log.emplace_back("recv", peer, n * 4);
    if (ipc != nullptr) {
      ipc->recv(p, n, peer, st);
      return;
    }
    const ncclResult_t r = ncclRecv(p, (size_t)n, ncclFloat32, peer, rccl->get(), st);
    TORCH_CHECK(r == ncclSuccess, "SplitEpoch: ncclRecv: ", ncclGetErrorString(r));
  }
};

class SplitEpoch {
 public:
  // cfg: mode (1 vanilla, 2 U-shape); B; role (0 = both sides here, 1 = the Alice only,
  // 2 = Bob only; remote roles also take peer and channel: an IpcChannel or a TpComm).
  // The Alice side: x (uint8 [N, 784]), y (int64 [N]); front {w, b} and front_opt; head {w, b}
  // (U-shape; Alice's optimizer).  Bob's side: tail (list of {w, b}) and bob_opt; p1, p2
  // (vanilla dropout); the workspaces.  Every parameter entry is {p, s0, s1}.
  explicit SplitEpoch(const py::dict& cfg) {
    mode_ = cfg["mode"].cast<int>();
    TORCH_CHECK(mode_ == 1 || mode_ == 2, "SplitEpoch: mode 1 (vanilla) or 2 (U-shape)");
    B_ = cfg["B"].cast<int>();
    TORCH_CHECK(B_ >= 1 && B_ <= 64, "SplitEpoch: batch 1..64 (the wgrad look-ahead's row range)");
    role_ = cfg.contains("role") ? cfg["role"].cast<int>() : 0;
    TORCH_CHECK(role_ >= 0 && role_ <= 2, "SplitEpoch: role 0 (both), 1 (Alice) or 2 (Bob)");
    const bool alice = role_ != 2, bob = role_ != 1;
    if (role_ != 0) {
      link_.peer = cfg["peer"].cast<int>();
      const py::object ch = cfg["channel"];
      if (py::isinstance<sl::IpcChannel>(ch)) {
        link_.ipc = ch.cast<sl::IpcChannel*>();
        TORCH_CHECK(link_.ipc->opened() && link_.ipc->cap() >= act_msg_words(B_),
                    "SplitEpoch: the peer-mapped channel is not open or too small for a batch");
      } else {
        link_.rccl = ch.cast<sl::TpComm*>();
      }
      channel_ = ch;    // keep the channel alive with the executor
    }
    at::Device dev = at::kCPU;
    if (alice) {
      x_ = get(cfg, "x");
      y_ = get(cfg, "y");
      TORCH_CHECK(x_.is_cuda() && x_.scalar_type() == at::kByte && x_.is_contiguous() && x_.numel() % 784 == 0,
                  "shard pixels uint8 [N, 784]");
      TORCH_CHECK(y_.is_cuda() && y_.scalar_type() == at::kLong && y_.is_contiguous() &&
                      y_.numel() == x_.numel() / 784,
                  "shard labels int64 [N]");
      const py::dict front = cfg["front"].cast<py::dict>();
      fw_ = read_param(front, "w");
      fb_ = read_param(front, "b");
      TORCH_CHECK(fw_.p.numel() == 288 && fb_.p.numel() == 32, "the 1 -> 32, 3 x 3 conv front");
      fopt_ = read_opt(cfg["front_opt"].cast<py::dict>());
      if (mode_ == 2) {
        const py::dict head = cfg["head"].cast<py::dict>();
        hw_ = read_param(head, "w");
        hb_ = read_param(head, "b");
        TORCH_CHECK(hw_.p.dim() == 2, "head W [C, 100]");
      }
      dev = x_.device();
    }
    if (bob) {
      bopt_ = read_opt(cfg["bob_opt"].cast<py::dict>());
      for (const auto& h : cfg["tail"].cast<std::vector<py::dict>>()) {
        L_.push_back({read_param(h, "w"), read_param(h, "b")});
        TORCH_CHECK(L_.back().w.p.dim() == 2 && L_.back().w.p.size(1) % 4 == 0, "tail W [N, K], K % 4 == 0");
      }
      const size_t nl = mode_ == 1 ? 3 : 2;
      TORCH_CHECK(L_.size() == nl, "SplitEpoch: vanilla drives model2_sisa (3 layers), U-shape model2 (2)");
      TORCH_CHECK(L_[0].w.p.size(1) == kCut, "fc1 takes the 5408-wide cut activation");
      for (size_t i = 1; i < nl; ++i) TORCH_CHECK(L_[i].w.p.size(1) == L_[i - 1].w.p.size(0), "tail chain shapes");
      p1_ = cfg["p1"].cast<double>();
      p2_ = cfg["p2"].cast<double>();
      dev = L_[0].w.p.device();
    }
    if (alice && bob && mode_ == 2)
      TORCH_CHECK(hw_.p.size(1) == L_[1].w.p.size(0), "head W [C, 100] on the middle's output");
    auto f32 = [&](int64_t n) { return at::empty({n}, at::TensorOptions().dtype(at::kFloat).device(dev)); };
    // the middle's / head's width: Bob's fc2 rows, or (the Alice alone) her head's input
    const int64_t N2 = bob ? L_[1].w.p.size(0) : (mode_ == 2 ? hw_.p.size(1) : 0);
    const int64_t N1 = bob ? L_[0].w.p.size(0) : 0;
    const int64_t Cl = mode_ == 1 ? (bob ? L_[2].w.p.size(0) : 0) : (alice ? hw_.p.size(0) : 0);
    for (int i = 0; i < 2; ++i) {
      // room for the vanilla message's label words behind the activation
      act_[i] = f32(act_msg_words(B_));
      if (alice) {
        am_[i] = at::empty({(int64_t)B_ * kCut}, at::TensorOptions().dtype(at::kByte).device(dev));
        lab_[i] = at::empty({(int64_t)B_}, at::TensorOptions().dtype(at::kLong).device(dev));
        slab_[i] = f32((int64_t)std::max(B_, 64) * 320);
      }
    }
    h2_ = f32(std::max<int64_t>(1, (int64_t)B_ * N2));
    dz2_ = f32(std::max<int64_t>(1, (int64_t)B_ * N2));
    dx_ = f32((int64_t)B_ * kCut);
    loss_ = f32((int64_t)B_);
    if (alice && mode_ == 2) {
      // Alice's head as one head_step launch (UShapeSession.head_fused)
      TORCH_CHECK((int64_t)B_ * N2 <= 4096 && (int64_t)B_ * Cl <= 1024 && Cl * N2 <= 4096,
                  "SplitEpoch: the U-shape head needs B * 100 <= 4096 (B <= 40)");
    }
    if (!bob) return;
    const int64_t S1 = (kCut + 255) / 256;
    pn_ = f32(S1 * B_ * N1);
    h1_ = f32((int64_t)B_ * N1);
    dz1_ = f32((int64_t)B_ * N1);
    dlog_ = f32(std::max<int64_t>(1, (int64_t)B_ * Cl));
    const int64_t nmax = std::max<int64_t>({N1, N2, Cl}), kmax = kCut;
    // the split-K / split-N workspaces: the caller's (ops/hip_ops.py `_workspace`, so every
    // split factor is the Python path's), at least that path's minimum sizes
    auto ws = [&](const char* k, int64_t n) {
      if (!cfg.contains(k)) return f32(n);
      at::Tensor t = get(cfg, k);
      need(t, k);
      TORCH_CHECK(t.numel() >= n, "SplitEpoch: workspace '", k, "' too small");
      return t;
    };
    fwdws_ = ws("fwdws", 16 * (int64_t)B_ * nmax);
    dgws_ = ws("dgws", 16 * (int64_t)B_ * kmax);
    if (mode_ == 1) {
      C3_ = (int)L_[2].w.p.size(0);
      p2ws_ = ws("p2ws", 16 * (int64_t)B_ * N2);
      headws_ = ws("headws", (int64_t)sl::head3_slices((int)N2) * B_ * C3_);
    }
  }

  // One epoch over order[0 .. n) (batches of B, last one partial).  t_a / t_b: the Alice and
  // Bob optimizer steps taken so far; fwd_count: Bob's forward counter (dropout hash).
  // Returns the updated (t_a, t_b, fwd_count).
  py::tuple run(const at::Tensor& order, int64_t t_a, int64_t t_b, int64_t fwd_count, int64_t seed_base) {
    TORCH_CHECK(role_ == 0, "SplitEpoch.run: both sides in this process (role 0)");
    const int64_t n = check_order(order);
    if (n == 0) return py::make_tuple(t_a, t_b, fwd_count);
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    const int64_t* ord = order.data_ptr<int64_t>();
    const int64_t T = (n + B_ - 1) / B_;
    auto rows = [&](int64_t i) { return (int)std::min<int64_t>(B_, n - i * B_); };
    pend_slab_ = -1;
    slab_i_ = 0;
    int cur = 0;
    alice_fwd(ord, rows(0), cur, lab_[cur].data_ptr<int64_t>(), st);
    bool pre = false;
    for (int64_t i = 0; i < T; ++i) {
      const int M = rows(i);
      ++fwd_count;
      float* act = act_[cur].data_ptr<float>();
      if (mode_ == 1)
        bob_vanilla(act, lab_[cur].data_ptr<int64_t>(), M, fwd_count, seed_base, pre, st);
      else
        t_a = bob_ushape(act, lab_[cur].data_ptr<int64_t>(), M, pre, t_a, st);
      pre = false;
      // Alice: dW partials of batch i (the kernel stores the pending update of batch i-1)
      if (mode_ == 1) ++t_a;
      alice_bwd(ord + i * B_, M, cur, t_a, st);
      // Alice: forward of batch i+1 (her update of batch i applied in-kernel)
      const bool more = i + 1 < T;
      if (more) alice_fwd(ord + (i + 1) * B_, rows(i + 1), cur ^ 1, lab_[cur ^ 1].data_ptr<int64_t>(), st);
      // Bob: grouped wgrad + optimizer, with batch i+1's fc1 product when it is <= 64 rows
      ++t_b;
      const float* xn = more ? act_[cur ^ 1].data_ptr<float>() : nullptr;
      bob_update(act, M, xn, more ? rows(i + 1) : 0, t_b, st);
      pre = xn != nullptr;
      cur ^= 1;
    }
    alice_flush(st);
    return py::make_tuple(t_a, t_b, fwd_count);
  }

  // The Alice's half of a remote epoch over order[0 .. n).  Returns her updated step count.
  int64_t run_alice(const at::Tensor& order, int64_t t_a) {
    TORCH_CHECK(role_ == 1, "SplitEpoch.run_alice: the Alice's side of a remote placement (role 1)");
    const int64_t n = check_order(order);
    if (n == 0) return t_a;
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    const int64_t* ord = order.data_ptr<int64_t>();
    const int64_t T = (n + B_ - 1) / B_;
    auto rows = [&](int64_t i) { return (int)std::min<int64_t>(B_, n - i * B_); };
    // vanilla: the labels ride in the activation message, behind the rows
    auto labs = [&](int buf, int M) {
      return mode_ == 1 ? reinterpret_cast<int64_t*>(act_[buf].data_ptr<float>() + (int64_t)M * kCut)
                        : lab_[buf].data_ptr<int64_t>();
    };
    const int N2 = mode_ == 2 ? (int)hw_.p.size(1) : 0, C = mode_ == 2 ? (int)hw_.p.size(0) : 0;
    pend_slab_ = -1;
    slab_i_ = 0;
    int cur = 0;
    alice_fwd(ord, rows(0), cur, labs(cur, rows(0)), st);
    for (int64_t i = 0; i < T; ++i) {
      const int M = rows(i);
      float* act = act_[cur].data_ptr<float>();
      if (mode_ == 1) {
        link_.send(act, act_msg_words(M), st);
        link_.recv(dx_.data_ptr<float>(), (int64_t)M * kCut, st);
        ++t_a;
      } else {
        link_.send(act, (int64_t)M * kCut, st);
        link_.recv(h2_.data_ptr<float>(), (int64_t)M * N2, st);
        ++t_a;
        // her head: forward + CE + d(mid) (masked by Bob's last ReLU) + the head update
        ck(sl::head_step(h2_.data_ptr<float>(), hw_.p.data_ptr<float>(), hb_.p.data_ptr<float>(),
                         lab_[cur].data_ptr<int64_t>(), -100, (float)(1.0 / M), loss_.data_ptr<float>(),
                         dz2_.data_ptr<float>(), hw_.s0, hw_.s1, hb_.s0, hb_.s1, M, N2, C, fopt_.at(t_a), true, st),
           "alice head step");
        link_.send(dz2_.data_ptr<float>(), (int64_t)M * N2, st);
        link_.recv(dx_.data_ptr<float>(), (int64_t)M * kCut, st);
      }
      alice_bwd(ord + i * B_, M, cur, t_a, st);
      if (i + 1 < T) alice_fwd(ord + (i + 1) * B_, rows(i + 1), cur ^ 1, labs(cur ^ 1, rows(i + 1)), st);
      cur ^= 1;
    }
    alice_flush(st);
    return t_a;
  }

  // Bob's half of a remote epoch of n samples.  Returns the updated (t_b, fwd_count).
  py::tuple run_bob(int64_t n, int64_t t_b, int64_t fwd_count, int64_t seed_base) {
    TORCH_CHECK(role_ == 2, "SplitEpoch.run_bob: Bob's side of a remote placement (role 2)");
    if (n <= 0) return py::make_tuple(t_b, fwd_count);
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    const int64_t T = (n + B_ - 1) / B_;
    const int N1 = (int)L_[0].w.p.size(0), N2 = (int)L_[1].w.p.size(0);
    float* act = act_[0].data_ptr<float>();
    for (int64_t i = 0; i < T; ++i) {
      const int M = (int)std::min<int64_t>(B_, n - i * B_);
      ++fwd_count;
      if (mode_ == 1) {
        link_.recv(act, act_msg_words(M), st);
        bob_vanilla(act, reinterpret_cast<const int64_t*>(act + (int64_t)M * kCut), M, fwd_count, seed_base, false,
                    st);
        link_.send(dx_.data_ptr<float>(), (int64_t)M * kCut, st);
      } else {
        link_.recv(act, (int64_t)M * kCut, st);
        fc1(act, M, sl::make_epi_raw(L_[0].b.p.data_ptr<float>(), true, 0.0, 0, 0, nullptr), false, st);
        ck(sl::linear_fwd(h1_.data_ptr<float>(), N1, L_[1].w.p.data_ptr<float>(), N1, h2_.data_ptr<float>(), N2, M,
                          N2, N1, sl::make_epi_raw(L_[1].b.p.data_ptr<float>(), true, 0.0, 0, 0, nullptr),
                          fwdws_.data_ptr<float>(), fwdws_.numel(), st),
           "fc2 forward");
        link_.send(h2_.data_ptr<float>(), (int64_t)M * N2, st);
        link_.recv(dz2_.data_ptr<float>(), (int64_t)M * N2, st);
        // d(mid) arrives premasked by the Alice's head step (UShapeSession.head_fused)
        ck(sl::linear_dgrad(dz2_.data_ptr<float>(), N2, L_[1].w.p.data_ptr<float>(), N1, h1_.data_ptr<float>(), N1,
                            1.f, dz1_.data_ptr<float>(), N1, dgws_.data_ptr<float>(), dgws_.numel(), M, N2, N1, st),
           "fc2 dgrad");
        cut_grad(M, st);
        link_.send(dx_.data_ptr<float>(), (int64_t)M * kCut, st);
      }
      // the update right after dx leaves: it runs during her backward and next forward
      ++t_b;
      bob_update(act, M, nullptr, 0, t_b, st);
    }
    return py::make_tuple(t_b, fwd_count);
  }

  // (op, peer, bytes) of every message this executor issued, in issue order
  std::vector<std::tuple<std::string, int, int64_t>> messages() const { return link_.log; }
  void clear_messages() { link_.log.clear(); }

 private:
  int64_t check_order(const at::Tensor& order) const {
    TORCH_CHECK(order.is_cuda() && order.scalar_type() == at::kLong && order.is_contiguous() && order.dim() == 1,
                "order int64 [n]");
    return order.numel();
  }

  // The Alice's deferred conv update: (slab, rows, step) of her last backward, not yet stored
  ConvPending pending() const {
    return ConvPending{slab_[pend_slab_].data_ptr<float>(), pend_rows_, fw_.s0, fw_.s1, fb_.s0, fb_.s1,
                       fopt_.at(pend_t_)};
  }

  // her conv forward of a batch into act_[buf] (gathers its labels into lab_out; applies the
  // pending update in-kernel)
  void alice_fwd(const int64_t* idx, int M, int buf, int64_t* lab_out, hipStream_t st) {
    const ConvPending p = pend_slab_ >= 0 ? pending() : ConvPending{};
    ck(sl::conv_fwd(x_.data_ptr(), true, idx, 0, M, fw_.p.data_ptr<float>(), fb_.p.data_ptr<float>(),
                    act_[buf].data_ptr<float>(), am_[buf].data_ptr<uint8_t>(), st, y_.data_ptr<int64_t>(), lab_out,
                    pend_slab_ >= 0 ? &p : nullptr),
       "alice conv forward");
  }

  // her conv backward from dx_: dW partials of this batch (the kernel stores the pending
  // update of the previous one); this batch's update becomes the pending one (step t)
  void alice_bwd(const int64_t* idx, int M, int buf, int64_t t, hipStream_t st) {
    const ConvPending p = pend_slab_ >= 0 ? pending() : ConvPending{};
    ck(sl::conv_bwd_step(dx_.data_ptr<float>(), act_[buf].data_ptr<float>(), am_[buf].data_ptr<uint8_t>(),
                         x_.data_ptr(), true, idx, M, fw_.p.data_ptr<float>(), fb_.p.data_ptr<float>(),
                         slab_[slab_i_].data_ptr<float>(), fw_.s0, fw_.s1, fb_.s0, fb_.s1, SlOpt{}, st, true,
                         pend_slab_ >= 0 ? &p : nullptr),
       "alice conv backward");
    pend_slab_ = slab_i_;
    pend_rows_ = M;
    pend_t_ = t;
    slab_i_ ^= 1;
  }

  // the last pending update (FrontEngine.flush)
  void alice_flush(hipStream_t st) {
    if (pend_slab_ < 0) return;
    ck(sl::conv_apply(pending(), fw_.p.data_ptr<float>(), fb_.p.data_ptr<float>(), st), "alice conv apply");
    pend_slab_ = -1;
  }

  // fc1 (+ReLU [+dropout]) of the batch: the look-ahead slabs' epilogue or a plain forward
  void fc1(const float* act, int M, const Epi& e1, bool pre, hipStream_t st) {
    const int N1 = (int)L_[0].w.p.size(0);
    if (pre)
      ck(sl::linear_epilogue(pn_.data_ptr<float>(), N1, h1_.data_ptr<float>(), N1, M, N1, e1, (kCut + 255) / 256,
                             (int64_t)M * N1, st),
         "fc1 epilogue");
    else
      ck(sl::linear_fwd(act, kCut, L_[0].w.p.data_ptr<float>(), kCut, h1_.data_ptr<float>(), N1, M, N1, kCut, e1,
                        fwdws_.data_ptr<float>(), fwdws_.numel(), st),
         "fc1 forward");
  }

  // dx = dz1 . W1 (the cut gradient for Alice)
  void cut_grad(int M, hipStream_t st) {
    const int N1 = (int)L_[0].w.p.size(0);
    ck(sl::linear_dgrad(dz1_.data_ptr<float>(), N1, L_[0].w.p.data_ptr<float>(), kCut, nullptr, 0, 1.f,
                        dx_.data_ptr<float>(), kCut, dgws_.data_ptr<float>(), dgws_.numel(), M, N1, kCut, st),
       "fc1 dgrad");
  }

  // vanilla: Bob's forward + CE + data gradients (TailEngine.train_fwd_bwd3, need_dx)
  void bob_vanilla(const float* act, const int64_t* lab, int M, int64_t fc, int64_t seed_base, bool pre,
                   hipStream_t st) {
    const int N1 = (int)L_[0].w.p.size(0), N2 = (int)L_[1].w.p.size(0);
    const uint64_t sd0 = sl::step_seed((uint64_t)seed_base, 0, (uint64_t)fc);
    const uint64_t sd1 = sl::step_seed((uint64_t)seed_base, 1, (uint64_t)fc);
    fc1(act, M, sl::make_epi_raw(L_[0].b.p.data_ptr<float>(), true, p1_, sd0, 0, nullptr), pre, st);
    int S2 = 1;
    ck(sl::linear_fwd_partial(h1_.data_ptr<float>(), N1, L_[1].w.p.data_ptr<float>(), N1, M, N2, N1,
                              p2ws_.data_ptr<float>(), p2ws_.numel(), 16, &S2, st),
       "fc2 forward");
    const Epi e2 = sl::make_epi_raw(L_[1].b.p.data_ptr<float>(), true, p2_, sd1, 0, nullptr);
    ck(sl::server_head3(p2ws_.data_ptr<float>(), S2, (int64_t)M * N2, e2, L_[2].w.p.data_ptr<float>(), N2,
                        L_[2].b.p.data_ptr<float>(), lab, -100, (float)(1.0 / M), h2_.data_ptr<float>(),
                        dlog_.data_ptr<float>(), dz2_.data_ptr<float>(), loss_.data_ptr<float>(),
                        headws_.data_ptr<float>(), headws_.numel(), M, N2, C3_, st),
       "server head");
    const float s1 = p1_ > 0 ? (float)(1.0 / (1.0 - p1_)) : 1.f;
    ck(sl::linear_dgrad(dz2_.data_ptr<float>(), N2, L_[1].w.p.data_ptr<float>(), N1, h1_.data_ptr<float>(), N1, s1,
                        dz1_.data_ptr<float>(), N1, dgws_.data_ptr<float>(), dgws_.numel(), M, N2, N1, st),
       "fc2 dgrad");
    cut_grad(M, st);
  }

  // U-shape: Bob's middle forward, Alice's head step, Bob's data gradients.  Returns Alice's
  // step count (the head and the front share the tick of this batch).
  int64_t bob_ushape(const float* act, const int64_t* lab, int M, bool pre, int64_t t_a, hipStream_t st) {
    const int N1 = (int)L_[0].w.p.size(0), N2 = (int)L_[1].w.p.size(0), C = (int)hw_.p.size(0);
    fc1(act, M, sl::make_epi_raw(L_[0].b.p.data_ptr<float>(), true, 0.0, 0, 0, nullptr), pre, st);
    ck(sl::linear_fwd(h1_.data_ptr<float>(), N1, L_[1].w.p.data_ptr<float>(), N1, h2_.data_ptr<float>(), N2, M, N2,
                      N1, sl::make_epi_raw(L_[1].b.p.data_ptr<float>(), true, 0.0, 0, 0, nullptr),
                      fwdws_.data_ptr<float>(), fwdws_.numel(), st),
       "fc2 forward");
    ++t_a;
    // Alice's head: forward + CE + dL/dmid (masked by Bob's last ReLU) + her head update
    ck(sl::head_step(h2_.data_ptr<float>(), hw_.p.data_ptr<float>(), hb_.p.data_ptr<float>(), lab, -100,
                     (float)(1.0 / M), loss_.data_ptr<float>(), dz2_.data_ptr<float>(), hw_.s0, hw_.s1, hb_.s0,
                     hb_.s1, M, N2, C, fopt_.at(t_a), true, st),
       "alice head step");
    ck(sl::linear_dgrad(dz2_.data_ptr<float>(), N2, L_[1].w.p.data_ptr<float>(), N1, h1_.data_ptr<float>(), N1, 1.f,
                        dz1_.data_ptr<float>(), N1, dgws_.data_ptr<float>(), dgws_.numel(), M, N2, N1, st),
       "fc2 dgrad");
    cut_grad(M, st);
    return t_a;
  }

  // Bob's grouped wgrad + optimizer (TailEngine.fused_step / group_step) with the look-ahead
  void bob_update(const float* act, int M, const float* xn, int mn, int64_t t, hipStream_t st) {
    sl::WgGroup g{};
    g.n = (int)L_.size();
    const float* dzs[3] = {dz1_.data_ptr<float>(), dz2_.data_ptr<float>(), dlog_.data_ptr<float>()};
    const float* As[3] = {act, h1_.data_ptr<float>(), h2_.data_ptr<float>()};
    for (int i = 0; i < g.n; ++i) {
      sl::WgDesc& d = g.d[i];
      Layer& L = L_[i];
      d.dz = dzs[i];
      d.ldz = (int)L.w.p.size(0);
      d.A = As[i];
      d.lda = (int)L.w.p.size(1);
      d.W = L.w.p.data_ptr<float>();
      d.ldw = (int)L.w.p.size(1);
      d.s0 = L.w.s0;
      d.s1 = L.w.s1;
      d.bias = L.b.p.data_ptr<float>();
      d.sb0 = L.b.s0;
      d.sb1 = L.b.s1;
      d.N = (int)L.w.p.size(0);
      d.K = (int)L.w.p.size(1);
    }
    if (xn != nullptr && mn <= 64) {
      g.xn = xn;
      g.ldxn = kCut;
      g.mn = mn;
      g.pn = pn_.data_ptr<float>();
    }
    ck(sl::wgrad_group(g, M, bopt_.at(t), st), "bob wgrad_group");
  }

  struct Layer {
    Param w, b;
  };
  int mode_ = 1, B_ = 16, C3_ = 0, role_ = 0;
  int pend_slab_ = -1, pend_rows_ = 0, slab_i_ = 0;
  int64_t pend_t_ = 0;
  Link link_;
  py::object channel_;
  double p1_ = 0, p2_ = 0;
  at::Tensor x_, y_;
  Param fw_, fb_, hw_, hb_;
  Opt fopt_, bopt_;
  std::vector<Layer> L_;
  at::Tensor act_[2], am_[2], lab_[2], slab_[2];
  at::Tensor pn_, h1_, h2_, dz1_, dz2_, dx_, dlog_, loss_, fwdws_, p2ws_, dgws_, headws_;
};

}  // namespace

void sl_register_split(py::module& m) {
  py::class_<SplitEpoch>(m, "SplitEpoch")
      .def(py::init<const py::dict&>())
      .def("run", &SplitEpoch::run, py::arg("order"), py::arg("t_a"), py::arg("t_b"), py::arg("fwd_count"),
           py::arg("seed_base"))
      .def("run_alice", &SplitEpoch::run_alice, py::arg("order"), py::arg("t_a"))
      .def("run_bob", &SplitEpoch::run_bob, py::arg("n"), py::arg("t_b"), py::arg("fwd_count"), py::arg("seed_base"))
      .def("messages", &SplitEpoch::messages)
      .def("clear_messages", &SplitEpoch::clear_messages);
}
