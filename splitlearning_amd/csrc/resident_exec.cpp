// Host side of the register-resident server epoch (`_C.ResidentEpoch`, csrc/resident.hip).
//
// Reference: bob.train_and_backward's inner loop (data_entities_vanilla_sisa.py:298-313).
// One `run` call = ONE launch over every full batch of a client's cached activations; the
// host precomputes the per-step Adam scalars (host.h make_opt_raw, bit-identical to the
// launch-per-stage executor's) and dropout seeds (host.h step_seed == ops/rng.py) as device
// tables, zeroes the arrival counters, launches, and reads the kernel's error word once.
// A trailing partial batch is left to the launch-per-stage executor (engine/tail.py).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <string>
#include <vector>

#include "host.h"
#include "resident.h"

namespace py = pybind11;

namespace {

at::Tensor get_t(const py::dict& d, const char* k) {
  TORCH_CHECK(d.contains(k) && !d[k].is_none(), "ResidentEpoch: missing '", k, "'");
  return d[k].cast<at::Tensor>();
}

struct LayerT {
  at::Tensor W, b, s0, s1, sb0, sb1;
};

class ResidentEpoch {
 public:
  // cfg: layers = [3 dicts {W, b, s0, s1, sb0, sb1}] (this shard's fc1 / fc2 / fc3 and
  // optimizer state), kind (2 = Adam, 1 = SGD-momentum), lr / beta1 / beta2 / eps / wd /
  // momentum, p1 / p2 (dropout), col_off1, B, ipc (IpcAllReduce or None: tensor-parallel
  // fc2), timeout_s (bound on every in-launch wait)
  explicit ResidentEpoch(const py::dict& cfg) {
    auto layers = cfg["layers"].cast<std::vector<py::dict>>();
    TORCH_CHECK(layers.size() == 3, "ResidentEpoch drives the 3-layer server tail");
    kind_ = cfg["kind"].cast<int>();
    TORCH_CHECK(kind_ == 1 || kind_ == 2, "SGD-momentum or Adam");
    for (int i = 0; i < 3; ++i) {
      LayerT& L = L_[i];
      const py::dict& d = layers[i];
      L.W = get_t(d, "W");
      L.b = get_t(d, "b");
      L.s0 = get_t(d, "s0");
      L.sb0 = get_t(d, "sb0");
      if (kind_ == 2) {
        L.s1 = get_t(d, "s1");
        L.sb1 = get_t(d, "sb1");
      }
      for (const at::Tensor* t : {&L.W, &L.b, &L.s0, &L.sb0, &L.s1, &L.sb1})
        if (t->defined())
          TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), "layer tensors: f32 GPU");
      TORCH_CHECK(L.W.dim() == 2 && L.s0.sizes() == L.W.sizes() && L.b.numel() == L.W.size(0), "layer shapes");
    }
    TORCH_CHECK(L_[1].W.size(1) == L_[0].W.size(0) && L_[2].W.size(1) == L_[1].W.size(0), "layer chain shapes");
    lr_ = cfg["lr"].cast<double>();
    beta1_ = cfg["beta1"].cast<double>();
    beta2_ = cfg["beta2"].cast<double>();
    eps_ = cfg["eps"].cast<double>();
    wd_ = cfg["wd"].cast<double>();
    mom_ = cfg["momentum"].cast<double>();
    p1_ = cfg["p1"].cast<double>();
    p2_ = cfg["p2"].cast<double>();
    col_off1_ = cfg["col_off1"].cast<int>();
    B_ = cfg["B"].cast<int>();
    if (cfg.contains("ipc") && !cfg["ipc"].is_none()) ipc_ = cfg["ipc"].cast<sl::IpcAllReduce*>();
    timeout_s_ = cfg.contains("timeout_s") ? cfg["timeout_s"].cast<double>() : 30.0;

    const at::Device dev = L_[0].W.device();
    dev_ = dev.index();
    int cus = 0;
    TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_) == hipSuccess, "CU count");
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_) != hipSuccess || khz <= 0) khz = 100000;
    clock_khz_ = khz;

    sl::ResArgs& a = a_;
    a = sl::ResArgs{};
    a.N1 = (int)L_[0].W.size(0);
    a.K1 = (int)L_[0].W.size(1);
    a.N2 = (int)L_[1].W.size(0);
    a.C = (int)L_[2].W.size(0);
    a.N1p = (a.N1 + 3) & ~3;
    a.C4 = (a.C + 3) & ~3;
    a.M = B_;
    // workgroups: one per CU (up to 256); a smaller count lets several ranks' persistent
    // launches share one GPU (the multi-process test, scripts/resident_tp_one_gpu.py)
    const int wg = cfg.contains("workgroups") ? cfg["workgroups"].cast<int>() : 0;
    a.G = wg > 0 ? std::min(wg, std::min(256, cus)) : std::min(256, cus);
    a.coop = wg > 0 ? 0 : 1;
    a.fault_step = -1;
    a.nrb = (a.N1 + 15) / 16;
    a.ncb = (a.K1 + 255) / 256;
    a.ngrp = (a.ncb + sl::kResTiles - 1) / sl::kResTiles;
    a.nfc1 = a.nrb * a.ngrp;
    a.ignore = -100;
    a.ce_scale = (float)(1.0 / B_);
    a.thr1 = p1_ > 0 ? (uint32_t)(p1_ * 4294967296.0) : 0u;
    a.thr2 = p2_ > 0 ? (uint32_t)(p2_ * 4294967296.0) : 0u;
    a.dsc1 = p1_ > 0 ? (float)(1.0 / (1.0 - p1_)) : 1.f;
    a.dsc2 = p2_ > 0 ? (float)(1.0 / (1.0 - p2_)) : 1.f;
    a.col_off1 = col_off1_;
    auto opt = at::TensorOptions().dtype(at::kFloat).device(dev);
    LA_ = at::zeros({2LL * a.ngrp * 16 * a.N1p}, opt);
    H1_ = at::zeros({2LL * 16 * a.N1p}, opt);
    LP_ = at::zeros({2LL * a.G * 16 * a.C4}, opt);
    DL_ = at::zeros({2LL * 16 * a.C4}, opt);
    DZ2_ = at::zeros({2LL * 16 * a.G * 4}, opt);
    W2B_ = at::zeros({2LL * a.nrb * a.G * 64}, opt);
    cnt_ = at::zeros({(int64_t)sl::kResCounters * sl::kResShardStride}, opt.dtype(at::kInt));
    err_ = at::zeros({1}, opt.dtype(at::kInt));
    // arrivals per counter shard (producer workgroup w lands on shard w % 8)
    std::vector<int> sn(sl::kResSeams * 8, 0);
    for (int w = 0; w < a.G; ++w) {
      if (w < a.nrb) ++sn[0 * 8 + (w & 7)];   // seam A: one arrival per row block (its last column group)
      ++sn[1 * 8 + (w & 7)];
      if (w < a.M) ++sn[2 * 8 + (w & 7)];
      ++sn[3 * 8 + (w & 7)];
    }
    shard_n_ = at::tensor(sn, at::TensorOptions().dtype(at::kInt)).to(dev);
    a.LA = LA_.data_ptr<float>();
    a.H1 = H1_.data_ptr<float>();
    a.LP = LP_.data_ptr<float>();
    a.DL = DL_.data_ptr<float>();
    a.DZ2 = DZ2_.data_ptr<float>();
    a.W2B = W2B_.data_ptr<float>();
    a.cnt = reinterpret_cast<unsigned*>(cnt_.data_ptr<int>());
    a.shard_n = shard_n_.data_ptr<int>();
    a.err = err_.data_ptr<int>();
    a.timeout = (int64_t)(timeout_s_ * 1000.0 * clock_khz_);
    auto setL = [](sl::ResLayer& r, LayerT& L) {
      r.W = L.W.data_ptr<float>();
      r.b = L.b.data_ptr<float>();
      r.m = L.s0.data_ptr<float>();
      r.mb = L.sb0.data_ptr<float>();
      r.v = L.s1.defined() ? L.s1.data_ptr<float>() : nullptr;
      r.vb = L.sb1.defined() ? L.sb1.data_ptr<float>() : nullptr;
    };
    setL(a.L1, L_[0]);
    setL(a.L2, L_[1]);
    setL(a.L3, L_[2]);
    a.o = sl::make_opt_raw(kind_, lr_, beta1_, beta2_, eps_, wd_, mom_, 0, nullptr);
    if (ipc_ != nullptr) {
      TORCH_CHECK(ipc_->opened(), "ResidentEpoch: the peer-mapped region is not open");
      TORCH_CHECK((int64_t)a.G * 64 * 2 <= ipc_->cap(),
                  "ResidentEpoch: peer-mapped region too small for the fc2 exchange");
    }
    std::string why;
    ok_ = sl::resident_fits(a, dev_, &why);
    why_ = why;
  }

  bool ok() const { return ok_; }
  std::string why() const { return why_; }
  int workgroups() const { return a_.G; }
  int clock_khz() const { return clock_khz_; }
  // tests: in the next run, step `step`'s first hand-off wait is never met (times out, err 2)
  void set_fault_step(int64_t step) { fault_step_ = step; }

  // Every full batch of acts [n, K1] / labels [n] (the first n - n % B rows) in ONE launch;
  // losses into loss_rows [n].  Returns (fwd_count, t, rows done).
  // step_rows (optional): rows of each step's batch (<= B; acts exactly S * B rows, short
  // batches zero-padded with ignored labels), as HybridEpoch::run.
  py::tuple run(const at::Tensor& acts, const at::Tensor& labels, at::Tensor& loss_rows, int64_t seed_base,
                int64_t fwd_count, int64_t t, const c10::optional<at::Tensor>& trace,
                const c10::optional<std::vector<int64_t>>& step_rows) {
    TORCH_CHECK(ok_, "ResidentEpoch: this shard does not fit: ", why_);
    TORCH_CHECK(acts.is_cuda() && acts.scalar_type() == at::kFloat && acts.dim() == 2 && acts.is_contiguous() &&
                    acts.size(1) == a_.K1,
                "acts [n, K1] contiguous f32");
    TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                    labels.numel() == acts.size(0),
                "labels int64 [n]");
    TORCH_CHECK(loss_rows.is_cuda() && loss_rows.scalar_type() == at::kFloat && loss_rows.numel() >= acts.size(0),
                "loss [n]");
    const int64_t S = acts.size(0) / B_;
    if (S == 0) return py::make_tuple(fwd_count, t, (int64_t)0);
    if (step_rows.has_value())
      TORCH_CHECK((int64_t)step_rows->size() == S && acts.size(0) == S * B_,
                  "step_rows: one row count per step, acts exactly S * B rows");
    // per-step tables: Adam {step_size, 1/sqrt(bc2)} at steps t+1 .. t+S and the two dropout
    // seeds at forward counts fwd_count+1 .. fwd_count+S
    std::vector<float> adam(4 * S, 0.f);
    std::vector<int32_t> seeds(4 * S);
    for (int64_t i = 0; i < S; ++i) {
      const SlOpt o = sl::make_opt_raw(kind_, lr_, beta1_, beta2_, eps_, wd_, mom_, t + 1 + i, nullptr);
      adam[4 * i] = o.step_size;
      adam[4 * i + 1] = o.inv_bc2_sqrt;
      const int64_t rows = step_rows.has_value() ? (*step_rows)[i] : B_;
      TORCH_CHECK(rows >= 1 && rows <= B_, "step_rows: 1 .. B rows per step");
      adam[4 * i + 2] = (float)(1.0 / (double)rows);
      const uint64_t s0 = sl::step_seed((uint64_t)seed_base, 0, (uint64_t)(fwd_count + 1 + i));
      const uint64_t s1 = sl::step_seed((uint64_t)seed_base, 1, (uint64_t)(fwd_count + 1 + i));
      seeds[4 * i] = (int32_t)(uint32_t)(s0 & 0xffffffffull);
      seeds[4 * i + 1] = (int32_t)(uint32_t)(s0 >> 32);
      seeds[4 * i + 2] = (int32_t)(uint32_t)(s1 & 0xffffffffull);
      seeds[4 * i + 3] = (int32_t)(uint32_t)(s1 >> 32);
    }
    const at::Device dev = acts.device();
    adam_ = at::from_blob(adam.data(), {4 * S}, at::TensorOptions().dtype(at::kFloat)).to(dev);
    seeds_ = at::from_blob(seeds.data(), {4 * S}, at::TensorOptions().dtype(at::kInt)).to(dev);
    sl::ResArgs a = a_;
    a.S = (int)S;
    a.X = acts.data_ptr<float>();
    a.Y = labels.data_ptr<int64_t>();
    a.loss = loss_rows.data_ptr<float>();
    a.adam = adam_.data_ptr<float>();
    a.seeds = reinterpret_cast<const uint32_t*>(seeds_.data_ptr<int32_t>());
    a.ipc.T = 0;
    if (ipc_ != nullptr) a.ipc = ipc_->begin_steps(S);
    a.trace = nullptr;
    a.trace_steps = 0;
    if (trace.has_value()) {
      TORCH_CHECK(trace->is_cuda() && trace->scalar_type() == at::kLong && trace->is_contiguous() &&
                      trace->numel() % 32 == 0,
                  "trace int64 [2, steps, 16]");
      a.trace = trace->data_ptr<int64_t>();
      a.trace_steps = (int)(trace->numel() / 32);
    }
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    // the executor's own error word starts clear on every launch: a wait that gave up in an
    // earlier run (whose exception the caller handled) must not make this launch give up
    TORCH_CHECK(hipMemsetAsync(a.err, 0, sizeof(int), st) == hipSuccess, "resident error word");
    a.fault_step = fault_step_ < S ? (int)fault_step_ : -1;
    fault_step_ = -1;                  // one injected fault per arming
    const hipError_t le = sl::resident_epoch_launch(a, st);
    TORCH_CHECK(le == hipSuccess, "resident epoch launch: ", hipGetErrorString(le));
    const int e = err_.item<int>();   // one sync per client epoch
    TORCH_CHECK(e == 0, "resident server epoch: an in-launch wait gave up (error word ", e,
                "; 2 = a seam timed out, 4 = the peer-mapped fc2 exchange failed)");
    return py::make_tuple(fwd_count + S, t + S, S * B_);
  }

 private:
  LayerT L_[3];
  int kind_ = 2, col_off1_ = 0, B_ = 16, dev_ = 0, clock_khz_ = 100000;
  double lr_ = 0, beta1_ = 0, beta2_ = 0, eps_ = 0, wd_ = 0, mom_ = 0, p1_ = 0, p2_ = 0, timeout_s_ = 30.0;
  sl::IpcAllReduce* ipc_ = nullptr;
  sl::ResArgs a_{};
  int64_t fault_step_ = -1;
  bool ok_ = false;
  std::string why_;
  at::Tensor LA_, H1_, LP_, DL_, DZ2_, W2B_, cnt_, err_, shard_n_, adam_, seeds_;
};

}  // namespace

void sl_register_resident(py::module& m) {
  py::class_<ResidentEpoch>(m, "ResidentEpoch")
      .def(py::init<const py::dict&>())
      .def("ok", &ResidentEpoch::ok)
      .def("set_fault_step", &ResidentEpoch::set_fault_step)
      .def("why", &ResidentEpoch::why)
      .def("workgroups", &ResidentEpoch::workgroups)
      .def("clock_khz", [](const ResidentEpoch& e) { return e.clock_khz(); })
      .def("run", &ResidentEpoch::run, py::arg("acts"), py::arg("labels"), py::arg("loss_rows"),
           py::arg("seed_base"), py::arg("fwd_count"), py::arg("t"), py::arg("trace") = py::none(),
           py::arg("step_rows") = py::none());
}
