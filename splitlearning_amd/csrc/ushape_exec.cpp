// Host side of the U-shape persistent split epoch (`_C.UShapeEpoch`, csrc/ushape.hip).
//
// Reference: the U-shape hot loop, data_entities.py:65-81.  One `run` call = one launch (or a
// few, `set_max_steps`) over every batch of a co-located Alice's epoch order, a short final batch
// included (padded to B rows with ignored labels and zero activations, its CE mean over its real
// rows).  The host builds the per-step tables (batch rows, labels, both sides' Adam step
// scalars: host.h make_opt_raw, as the per-batch executor; CE scales), zeroes the counters (in
// the launch), launches and reads the kernel's error word once per launch.
//
// Remote Alice (cfg channel / peer / G; BASELINE config 2 on two GPUs): `run_remote` is Bob's side
// of her epoch as one launch exchanging run_bob's four messages per step on the peer-mapped channel
// itself (csrc/ushape.hip REM); her side stays csrc/split.cpp run_alice.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <string>
#include <tuple>
#include <vector>

#include "host.h"
#include "ipc_p2p.h"
#include "ushape.h"

namespace py = pybind11;

namespace {

at::Tensor us_get(const py::dict& d, const char* k) {
  TORCH_CHECK(d.contains(k) && !d[k].is_none(), "UShapeEpoch: missing '", k, "'");
  at::Tensor t = d[k].cast<at::Tensor>();
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "UShapeEpoch: '", k, "' f32 GPU");
  return t;
}

struct Six {
  at::Tensor W, m, v, b, mb, vb;
};

Six us_six(const py::dict& d) {
  Six s{us_get(d, "W"), us_get(d, "m"), us_get(d, "v"), us_get(d, "b"), us_get(d, "mb"), us_get(d, "vb")};
  TORCH_CHECK(s.m.sizes() == s.W.sizes() && s.v.sizes() == s.W.sizes() && s.mb.numel() == s.b.numel() &&
                  s.vb.numel() == s.b.numel(),
              "UShapeEpoch: parameter / moment shapes");
  return s;
}

SlOpt us_opt(const py::dict& d, int64_t t) {
  return sl::make_opt_raw(2, d["lr"].cast<double>(), d["beta1"].cast<double>(), d["beta2"].cast<double>(),
                          d["eps"].cast<double>(), d["wd"].cast<double>(), 0.0, t, nullptr);
}

class UShapeEpoch {
 public:
  // cfg: fc1 / fc2 (Bob's model2) and conv / head (Alice's model1 / model3), each {W, m, v, b,
  // mb, vb} (conv W [32, 1, 3, 3]); bob_opt / alice_opt {lr, beta1, beta2, eps, wd}; x (uint8
  // shard [N, 784]), y (int64 labels [N]); B; timeout_s; workgroups (0: cooperative launch)
  // Remote Alice: channel (an open IpcChannel), peer (her rank) and G (32 per 128-row fc1 group;
  // default 256) in place of conv / head / alice_opt / x / y.
  explicit UShapeEpoch(const py::dict& cfg) {
    f1_ = us_six(cfg["fc1"].cast<py::dict>());
    f2_ = us_six(cfg["fc2"].cast<py::dict>());
    bo_ = cfg["bob_opt"].cast<py::dict>();
    rem_ = cfg.contains("channel") && !cfg["channel"].is_none();
    if (rem_) {
      const py::object ch = cfg["channel"];
      TORCH_CHECK(py::isinstance<sl::IpcChannel>(ch), "UShapeEpoch: channel must be an IpcChannel");
      chan_ = ch.cast<sl::IpcChannel*>();
      channel_ = ch;
      peer_ = cfg["peer"].cast<int>();
      TORCH_CHECK(chan_->opened() && peer_ >= 0 && peer_ < chan_->size() && peer_ != chan_->rank(),
                  "UShapeEpoch: an open channel and the Alice's rank");
      ao_ = bo_;
    } else {
      cv_ = us_six(cfg["conv"].cast<py::dict>());
      hd_ = us_six(cfg["head"].cast<py::dict>());
      ao_ = cfg["alice_opt"].cast<py::dict>();
      x_ = cfg["x"].cast<at::Tensor>();
      y_ = cfg["y"].cast<at::Tensor>();
      TORCH_CHECK(x_.is_cuda() && x_.scalar_type() == at::kByte && x_.is_contiguous() && x_.numel() % 784 == 0,
                  "shard pixels uint8 [N, 784]");
      TORCH_CHECK(y_.is_cuda() && y_.scalar_type() == at::kLong && y_.numel() * 784 == x_.numel(), "labels int64 [N]");
    }
    B_ = cfg["B"].cast<int>();
    timeout_s_ = cfg.contains("timeout_s") ? cfg["timeout_s"].cast<double>() : 30.0;
    const int wg = cfg.contains("workgroups") ? cfg["workgroups"].cast<int>() : 0;
    dev_ = f1_.W.device().index();
    int cus = 0, khz = 0;
    TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_) == hipSuccess, "CU count");
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_) != hipSuccess || khz <= 0) khz = 100000;

    sl::UsArgs& a = a_;
    a = sl::UsArgs{};
    a.N1 = (int)f1_.W.size(0);
    a.N2 = (int)f2_.W.size(0);
    a.C = rem_ ? 1 : (int)hd_.W.size(0);
    a.rem = rem_ ? 1 : 0;
    a.G = rem_ && cfg.contains("G") ? cfg["G"].cast<int>() : sl::kUsG;
    a.RG = a.G / 32;
    a.M = B_;
    a.coop = wg > 0 ? 0 : 1;
    a.bf16 = cfg.contains("bf16") && cfg["bf16"].cast<bool>() ? 1 : 0;
    a.fault_step = -1;
    a.ignore = -100;
    a.ob = us_opt(bo_, 1);
    a.oa = us_opt(ao_, 1);
    if (f1_.W.dim() != 2 || f1_.W.size(1) != sl::kUsCh * sl::kUsP) why_ = "fc1 input width 5408 (32 x 13 x 13)";
    else if (f2_.W.dim() != 2 || f2_.W.size(1) != a.N1) why_ = "fc2 input width = fc1 width";
    else if (!rem_ && (hd_.W.dim() != 2 || hd_.W.size(1) != a.N2)) why_ = "head input width = fc2 width";
    else if (!rem_ && (cv_.W.numel() != 288 || cv_.b.numel() != 32)) why_ = "conv 32 x 1 x 3 x 3";
    else if (cus < (rem_ ? a.G : sl::kUsG)) why_ = "fewer CUs than workgroups";
    else if (rem_ && chan_->cap() < (int64_t)B_ * sl::kUsCh * sl::kUsP) why_ = "the channel is too small for a batch";
    else {
      if (rem_) {   // placeholders the check requires; the launch's own are set per chunk
        a.lk.sdata[0] = reinterpret_cast<float*>(16);
        a.lk.rdata[0] = reinterpret_cast<const float*>(16);
      }
      why_ = sl::ushape_check(a);
    }
    if (why_.empty()) {
      auto opt = at::TensorOptions().dtype(at::kFloat).device(f1_.W.device());
      int64_t off = 0;
      auto take = [&](int64_t n) {
        const int64_t o = off;
        off += (n + 3) & ~3LL;
        return (int)o;
      };
      a.oXS = take(2LL * sl::kUsCh * 16 * sl::kUsKP);
      a.oPP = take(2LL * sl::kUsRG * sl::kUsCh * 128 * 16);
      a.oP2 = take(2LL * sl::kUsN2P * sl::kUsG * 16);
      a.oH2 = take(2LL * sl::kUsN2P * 16);
      a.oDL = take(2LL * 16 * sl::kUsCP);
      a.oDZ = take(2LL * sl::kUsRG * 128 * 16);
      a.oDX = take(2LL * sl::kUsCh * sl::kUsRG * sl::kUsKP * 16);
      a.oCW = take(2LL * sl::kUsCh * sl::kUsRG * 16);
      HB_ = at::zeros({off}, opt);   // padding columns / rows of the hand-offs stay zero
      cnt_ = at::zeros({(int64_t)sl::kUsCounters * sl::kUsStride}, opt.dtype(at::kInt));
      err_ = at::zeros({1}, opt.dtype(at::kInt));
      a.HB = HB_.data_ptr<float>();
      a.cnt = reinterpret_cast<unsigned*>(cnt_.data_ptr<int>());
      a.err = err_.data_ptr<int>();
      a.timeout = (int64_t)(timeout_s_ * 1000.0 * khz);
      auto set6 = [](const Six& s, float*& W, float*& m, float*& v, float*& b, float*& mb, float*& vb) {
        W = s.W.data_ptr<float>();
        m = s.m.data_ptr<float>();
        v = s.v.data_ptr<float>();
        b = s.b.data_ptr<float>();
        mb = s.mb.data_ptr<float>();
        vb = s.vb.data_ptr<float>();
      };
      set6(f1_, a.W1, a.m1, a.v1, a.b1, a.mb1, a.vb1);
      set6(f2_, a.W2, a.m2, a.v2, a.b2, a.mb2, a.vb2);
      if (!rem_) {
        set6(cv_, a.cw, a.cmw, a.cvw, a.cb, a.cmb, a.cvb);
        set6(hd_, a.W3, a.m3, a.v3, a.b3, a.mb3, a.vb3);
        a.img = x_.data_ptr<uint8_t>();
      }
      std::string why;
      sl::ushape_fits(a, dev_, &why);
      why_ = why;
    }
    ok_ = why_.empty();
  }

  bool ok() const { return ok_; }
  std::string why() const { return why_; }
  void set_fault_step(int64_t s) { fault_step_ = s; }
  void set_max_steps(int64_t s) { max_steps_ = std::max<int64_t>(1, s); }

  // One epoch over `order` (int64 shard rows [n] on the device): ceil(n / B) steps.  Per-row
  // losses -> loss_rows [>= S * B] (padding rows 0).  t_a / t_b: Alice's / Bob's Adam steps so
  // far.  Returns both advanced by the step count.  Raises when an in-launch wait gave up.
  py::tuple run(const at::Tensor& order, at::Tensor& loss_rows, int64_t t_a, int64_t t_b) {
    TORCH_CHECK(ok_, "UShapeEpoch: ", why_);
    TORCH_CHECK(!rem_, "UShapeEpoch.run: a co-located Alice (run_remote serves a remote one)");
    TORCH_CHECK(order.is_cuda() && order.scalar_type() == at::kLong && order.dim() == 1, "order int64 [n] on the GPU");
    const int64_t n = order.numel();
    const int64_t S = (n + B_ - 1) / B_;
    if (S == 0) return py::make_tuple(t_a, t_b);
    TORCH_CHECK(loss_rows.is_cuda() && loss_rows.scalar_type() == at::kFloat && loss_rows.numel() >= S * B_,
                "loss_rows f32 [>= S * B]");
    const at::Device dev = order.device();
    auto lopt = at::TensorOptions().dtype(at::kLong).device(dev);
    rows_ = at::full({S * B_}, -1, lopt);
    rows_.narrow(0, 0, n).copy_(order);
    labels_ = at::full({S * B_}, -100, lopt);
    labels_.narrow(0, 0, n).copy_(y_.index_select(0, order));
    std::vector<float> tabf(8 * S, 0.f);
    for (int64_t i = 0; i < S; ++i) {
      const SlOpt ob = us_opt(bo_, t_b + 1 + i), oa = us_opt(ao_, t_a + 1 + i);
      tabf[8 * i] = ob.step_size;
      tabf[8 * i + 1] = ob.inv_bc2_sqrt;
      tabf[8 * i + 2] = oa.step_size;
      tabf[8 * i + 3] = oa.inv_bc2_sqrt;
      tabf[8 * i + 4] = (float)(1.0 / (double)std::min<int64_t>(B_, n - i * B_));
      tabf[8 * i + 5] = (float)std::min<int64_t>(B_, n - i * B_);
    }
    tabf_ = at::from_blob(tabf.data(), {8 * S}, at::TensorOptions().dtype(at::kFloat)).to(dev);
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    TORCH_CHECK(hipMemsetAsync(a_.err, 0, sizeof(int), st) == hipSuccess, "U-shape error word");
    const int64_t cs = std::min<int64_t>(S, max_steps_);
    for (int64_t s0 = 0; s0 < S; s0 += cs) {
      if (s0 > 0 && err_.item<int>() != 0) break;   // a failed chunk stops the epoch
      const int64_t ns = std::min(cs, S - s0);
      sl::UsArgs a = a_;
      a.S = (int)ns;
      a.rows = rows_.data_ptr<int64_t>() + s0 * B_;
      a.Y = labels_.data_ptr<int64_t>() + s0 * B_;
      a.loss = loss_rows.data_ptr<float>() + s0 * B_;
      a.tabf = tabf_.data_ptr<float>() + 8 * s0;
      a.fault_step = fault_step_ >= s0 && fault_step_ < s0 + ns ? (int)(fault_step_ - s0) : -1;
      const hipError_t le = sl::ushape_epoch_launch(a, st);
      TORCH_CHECK(le == hipSuccess, "U-shape epoch launch: ", hipGetErrorString(le));
    }
    fault_step_ = -1;
    const int e = err_.item<int>();
    TORCH_CHECK(e == 0, "U-shape split epoch: an in-launch wait gave up (error word ", e, ")");
    return py::make_tuple(t_a + S, t_b + S);
  }

  // Bob's side of a remote Alice's epoch of n samples (her side: csrc/split.cpp run_alice): per
  // step her activation in, h2 out, her dz2 in, the cut gradient out, from inside the launch, in
  // run_bob's order and sizes.  Returns t_b advanced by the step count.  Fail-stop: raises when an
  // in-launch wait gave up.
  int64_t run_remote(int64_t n, int64_t t_b) {
    TORCH_CHECK(ok_, "UShapeEpoch: ", why_);
    TORCH_CHECK(rem_, "UShapeEpoch.run_remote: configured with a channel and peer");
    const int64_t S = n > 0 ? (n + B_ - 1) / B_ : 0;
    if (S == 0) return t_b;
    const at::Device dev = f1_.W.device();
    auto rows_at = [&](int64_t i) { return std::min<int64_t>(B_, n - i * B_); };
    std::vector<float> tabf(8 * S, 0.f);
    for (int64_t i = 0; i < S; ++i) {
      const SlOpt ob = us_opt(bo_, t_b + 1 + i);
      tabf[8 * i] = ob.step_size;
      tabf[8 * i + 1] = ob.inv_bc2_sqrt;
      tabf[8 * i + 4] = (float)(1.0 / (double)rows_at(i));
      tabf[8 * i + 5] = (float)rows_at(i);
    }
    tabf_ = at::from_blob(tabf.data(), {8 * S}, at::TensorOptions().dtype(at::kFloat)).to(dev);
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    TORCH_CHECK(hipMemsetAsync(a_.err, 0, sizeof(int), st) == hipSuccess, "U-shape error word");
    const int64_t cs = std::min<int64_t>(S, max_steps_);
    const int64_t N2 = a_.N2, cut = (int64_t)sl::kUsCh * sl::kUsP;
    log_.clear();
    for (int64_t s0 = 0; s0 < S; s0 += cs) {
      if (s0 > 0 && err_.item<int>() != 0) break;
      const int64_t ns = std::min(cs, S - s0);
      std::vector<int64_t> sends, recvs;
      for (int64_t i = s0; i < s0 + ns; ++i) {
        const int64_t M = rows_at(i);
        recvs.push_back(M * cut);
        recvs.push_back(M * N2);
        sends.push_back(M * N2);
        sends.push_back(M * cut);
        log_.emplace_back("recv", peer_, M * cut * 4);
        log_.emplace_back("send", peer_, M * N2 * 4);
        log_.emplace_back("recv", peer_, M * N2 * 4);
        log_.emplace_back("send", peer_, M * cut * 4);
      }
      const sl::P2PRun r = chan_->run(peer_, st, sends, recvs);
      sl::UsArgs a = a_;
      a.S = (int)ns;
      for (int p = 0; p < 2; ++p) {
        a.lk.sdata[p] = r.sdata[p];
        a.lk.sflag[p] = r.sflag[p];
        a.lk.sack[p] = r.sack[p];
        a.lk.rdata[p] = r.rdata[p];
        a.lk.rflag[p] = r.rflag[p];
        a.lk.rack[p] = r.rack[p];
        a.lk.sprev[p] = r.sprev[p];
      }
      a.lk.sgen0 = r.sgen0;
      a.lk.rgen0 = r.rgen0;
      a.lk.err = r.err;
      a.lk.herr = r.herr;
      a.tabf = tabf_.data_ptr<float>() + 8 * s0;
      a.fault_step = fault_step_ >= s0 && fault_step_ < s0 + ns ? (int)(fault_step_ - s0) : -1;
      const hipError_t le = sl::ushape_epoch_launch(a, st);
      TORCH_CHECK(le == hipSuccess, "U-shape epoch launch: ", hipGetErrorString(le));
    }
    fault_step_ = -1;
    const int e = err_.item<int>();
    TORCH_CHECK(e == 0, "U-shape remote split epoch: an in-launch wait gave up (error word ", e, ")");
    return t_b + S;
  }

  std::vector<std::tuple<std::string, int, int64_t>> messages() const { return log_; }
  bool remote() const { return rem_; }
  int workgroups() const { return rem_ ? a_.G : sl::kUsG; }

 private:
  bool rem_ = false;
  sl::IpcChannel* chan_ = nullptr;
  py::object channel_;
  int peer_ = -1;
  std::vector<std::tuple<std::string, int, int64_t>> log_;
  Six f1_, f2_, cv_, hd_;
  py::dict bo_, ao_;
  at::Tensor x_, y_, HB_, cnt_, err_, rows_, labels_, tabf_;
  int B_ = 16, dev_ = 0;
  double timeout_s_ = 30.0;
  int64_t fault_step_ = -1, max_steps_ = INT64_MAX / 4;
  sl::UsArgs a_{};
  bool ok_ = false;
  std::string why_;
};

}  // namespace

void sl_register_ushape(py::module& m) {
  py::class_<UShapeEpoch>(m, "UShapeEpoch")
      .def(py::init<const py::dict&>())
      .def("ok", &UShapeEpoch::ok)
      .def("why", &UShapeEpoch::why)
      .def("set_fault_step", &UShapeEpoch::set_fault_step)
      .def("set_max_steps", &UShapeEpoch::set_max_steps)
      .def("run", &UShapeEpoch::run, py::arg("order"), py::arg("loss_rows"), py::arg("t_a"), py::arg("t_b"))
      .def("run_remote", &UShapeEpoch::run_remote, py::arg("n"), py::arg("t_b"))
      .def("messages", &UShapeEpoch::messages)
      .def("remote", &UShapeEpoch::remote)
      .def("workgroups", &UShapeEpoch::workgroups);
}
