// Host side of the hybrid persistent server epoch (`_C.HybridEpoch`, csrc/hybrid.hip).
//
// Reference: bob.train_and_backward's inner loop (data_entities_vanilla_sisa.py:298-313).
// One `run` call = ONE launch over every full batch of a client's cached activations (a
// trailing partial batch is left to the launch-per-stage executor, engine/tail.py).  The host
// precomputes the per-step Adam scalars (host.h make_opt_raw, bit-identical to the launch-per-
// stage executor's) and dropout seeds (host.h step_seed == ops/rng.py) as device tables, the
// fc1 tile runs of the workgroups and the counters' arrival counts, zeroes the counters (in
// the launch), launches cooperatively and reads the kernel's error word once.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <string>
#include <vector>

#include "host.h"
#include "hybrid.h"

namespace py = pybind11;

namespace {

at::Tensor hy_get(const py::dict& d, const char* k) {
  TORCH_CHECK(d.contains(k) && !d[k].is_none(), "HybridEpoch: missing '", k, "'");
  return d[k].cast<at::Tensor>();
}

struct HyLayer {
  at::Tensor W, b, s0, s1, sb0, sb1;
};

class HybridEpoch {
 public:
  // cfg: layers = [3 dicts {W, b, s0, s1, sb0, sb1}], kind (2 Adam, 1 SGD-momentum), lr /
  // beta1 / beta2 / eps / wd / momentum, p1 / p2, col_off1, B, ipc (IpcAllReduce or None),
  // timeout_s, workgroups (0: one per CU, a multiple of 8)
  explicit HybridEpoch(const py::dict& cfg) {
    auto layers = cfg["layers"].cast<std::vector<py::dict>>();
    TORCH_CHECK(layers.size() == 3, "HybridEpoch drives the 3-layer server tail");
    kind_ = cfg["kind"].cast<int>();
    TORCH_CHECK(kind_ == 1 || kind_ == 2, "SGD-momentum or Adam");
    for (int i = 0; i < 3; ++i) {
      HyLayer& L = L_[i];
      const py::dict& d = layers[i];
      L.W = hy_get(d, "W");
      L.b = hy_get(d, "b");
      L.s0 = hy_get(d, "s0");
      L.sb0 = hy_get(d, "sb0");
      if (kind_ == 2) {
        L.s1 = hy_get(d, "s1");
        L.sb1 = hy_get(d, "sb1");
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

    sl::HyArgs& a = a_;
    a = sl::HyArgs{};
    a.N1 = (int)L_[0].W.size(0);
    a.K1 = (int)L_[0].W.size(1);
    a.N2 = (int)L_[1].W.size(0);
    a.C = (int)L_[2].W.size(0);
    a.C4 = (a.C + 3) & ~3;
    a.M = B_;
    const int wg = cfg.contains("workgroups") ? cfg["workgroups"].cast<int>() : 0;
    int G = std::min(wg > 0 ? wg : 256, std::min(256, cus));
    G -= G % sl::kHyNR;
    a.G = G;
    a.coop = wg > 0 ? 0 : 1;
    a.fault_step = -1;
    // steps per launch: the inputs of one launch are addressed with 32-bit buffer offsets
    // (S * M * K1 * 4 < 2 GB); cfg "chunk_steps" lowers the bound (tests)
    max_steps_ = (int64_t)(2147483647LL / ((int64_t)std::max(B_, 1) * std::max<int64_t>(L_[0].W.size(1), 1) * 4));
    if (cfg.contains("chunk_steps") && !cfg["chunk_steps"].is_none())
      max_steps_ = std::max<int64_t>(1, std::min<int64_t>(max_steps_, cfg["chunk_steps"].cast<int64_t>()));
    // fc1 state cache policy: the over-cache form (W plain, m / v non-temporal) when the
    // shard's streamed state is larger than the 256 MB Infinity Cache (TP = 1), write-through
    // when it fits (csrc/hybrid.hip kStW ..); cfg "nt_stores" (0 / 1) overrides for the A/B
    {
      const int64_t state = (int64_t)L_[0].W.numel() * 4 * (kind_ == 2 ? 3 : 2);
      const int o = cfg.contains("nt_stores") && !cfg["nt_stores"].is_none() ? cfg["nt_stores"].cast<int>() : -1;
      a.ntst = o >= 0 ? o : (state > (256LL << 20) ? 1 : 0);
    }
    a.NC = G / sl::kHyNR;
    a.HW = a.N2 / 4;
    a.nrb = (a.N1 + 15) / 16;
    a.ncb = (a.K1 + 255) / 256;
    a.ntile = a.nrb * a.ncb;
    a.ignore = -100;
    a.ce_scale = (float)(1.0 / B_);
    a.thr1 = p1_ > 0 ? (uint32_t)(p1_ * 4294967296.0) : 0u;
    a.thr2 = p2_ > 0 ? (uint32_t)(p2_ * 4294967296.0) : 0u;
    a.dsc1 = p1_ > 0 ? (float)(1.0 / (1.0 - p1_)) : 1.f;
    a.dsc2 = p2_ > 0 ? (float)(1.0 / (1.0 - p2_)) : 1.f;
    a.col_off1 = col_off1_;
    why_ = G < 8 ? "fewer than 8 CUs" : "";
    if (why_.empty()) why_ = tables();
    auto opt = at::TensorOptions().dtype(at::kFloat).device(dev);
    if (why_.empty()) {
      // the hand-off arena (offsets in floats, 16-B aligned)
      int64_t off = 0;
      auto take = [&](int64_t n) {
        const int64_t o = off;
        off += (n + 3) & ~3LL;
        return (int)o;
      };
      a.oLA = take(2LL * a.nrb * sl::kHySlots * 256);
      a.oH1 = take(2LL * 16 * a.N1);
      a.oFP = take(2LL * a.NC * 16 * a.N2);
      a.oLP = take(2LL * a.HW * 16 * a.C4);
      a.oDL = take(2LL * 16 * a.C4);
      a.oDZ = take(2LL * 16 * a.N2);
      a.oDP = take(2LL * sl::kHyNR * 16 * a.N1);
      a.oZP = take((int64_t)G * sl::kHyRuns * 8 * 64 * 4);
      HB_ = at::zeros({off}, opt);
      a.HB = HB_.data_ptr<float>();
      cnt_ = at::zeros({(int64_t)sl::kHyCounters * sl::kHyStride}, opt.dtype(at::kInt));
      err_ = at::zeros({1}, opt.dtype(at::kInt));
      std::vector<int> sn(sl::kHySeams * 8, 0);
      for (int w = 0; w < G; ++w) {
        ++sn[0 * 8 + (w & 7)];                 // F: every tile
        if (w < a.HW) ++sn[1 * 8 + (w & 7)];   // L: head workgroups
        if (w < a.M) ++sn[2 * 8 + (w & 7)];    // D: softmax workgroups
        if (w < a.HW) ++sn[3 * 8 + (w & 7)];   // Z: head workgroups
      }
      shard_n_ = at::tensor(sn, at::TensorOptions().dtype(at::kInt)).to(dev);
      a.cnt = reinterpret_cast<unsigned*>(cnt_.data_ptr<int>());
      a.shard_n = shard_n_.data_ptr<int>();
      a.err = err_.data_ptr<int>();
      a.tab = tab_.data_ptr<int>();
      a.timeout = (int64_t)(timeout_s_ * 1000.0 * clock_khz_);
      auto setL = [](sl::ResLayer& r, HyLayer& L) {
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
        TORCH_CHECK(ipc_->opened(), "HybridEpoch: the peer-mapped region is not open");
        a.ipc.T = ipc_->size();
        a.ipc.cap = ipc_->cap();
      }
      std::string why;
      sl::hybrid_fits(a, dev_, &why);
      why_ = why;
      a.ipc = sl::IpcStep{};
    }
    ok_ = why_.empty();
  }

  bool ok() const { return ok_; }
  std::string why() const { return why_; }
  int workgroups() const { return a_.G; }

  // Every full batch of acts [n, K1] / labels [n] (the first n - n % B rows): ONE launch, or
  // consecutive launches of at most max_steps_ steps when the epoch's inputs exceed the 32-bit
  // buffer offsets (each launch re-forms its first step's fc1 product in its prologue; one
  // launch of S steps is bitwise S one-step launches, tests/test_hybrid_gpu.py, so the chunked
  // epoch is bitwise the single launch).  Losses into loss_rows [n].  Returns (fwd_count, t,
  // rows done).  Raises when an in-launch wait gave up (the shard's state is then partly
  // updated: the caller restores it, protocols/sisa.py).
  //
  // step_rows (optional, [S] host ints): the batch of step i holds step_rows[i] <= B real rows
  // (its CE mean is over them); acts / labels are then exactly S * B rows, every short batch
  // zero-padded with ignored labels (-100), so every step of a whole server epoch over all
  // clients' caches, short final batches included, runs in the same launch (padded rows add
  // exact zeros to every gradient).
  py::tuple run(const at::Tensor& acts, const at::Tensor& labels, at::Tensor& loss_rows, int64_t seed_base,
                int64_t fwd_count, int64_t t, const c10::optional<at::Tensor>& trace,
                const c10::optional<at::Tensor>& trace_all, int64_t trace_all_step,
                const c10::optional<std::vector<int64_t>>& step_rows) {
    TORCH_CHECK(ok_, "HybridEpoch: this shard does not fit: ", why_);
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
    int64_t* tr = nullptr;
    int trs = 0;
    if (trace.has_value()) {
      TORCH_CHECK(trace->is_cuda() && trace->scalar_type() == at::kLong && trace->is_contiguous() &&
                      trace->numel() % 32 == 0,
                  "trace int64 [2, steps, 16]");
      tr = trace->data_ptr<int64_t>();
      trs = (int)(trace->numel() / 32);
    }
    int64_t* ta = nullptr;
    int tan = 0;
    if (trace_all.has_value()) {
      TORCH_CHECK(trace_all->is_cuda() && trace_all->scalar_type() == at::kLong && trace_all->is_contiguous() &&
                      trace_all->numel() >= 16LL * a_.G && trace_all->numel() % (16LL * a_.G) == 0,
                  "trace_all int64 [steps, G, 16]");
      ta = trace_all->data_ptr<int64_t>();
      tan = (int)(trace_all->numel() / (16LL * a_.G));
    }
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    // one clear of the error word per epoch; a chunk whose wait gave up leaves it set, and the
    // host reads it before issuing the next chunk (one sync per chunk of thousands of steps), so
    // no later chunk runs on a half-updated shard (the kernels only read the word inside a wait
    // that is not already met, so they cannot be relied on to stop by themselves)
    TORCH_CHECK(hipMemsetAsync(a_.err, 0, sizeof(int), st) == hipSuccess, "hybrid error word");
    const int64_t cs = std::max<int64_t>(1, max_steps_);
    for (int64_t s0 = 0; s0 < S; s0 += cs) {
      if (s0 > 0 && err_.item<int>() != 0) break;
      const int64_t n = std::min(cs, S - s0);
      sl::HyArgs a = a_;
      a.S = (int)n;
      a.X = acts.data_ptr<float>() + s0 * B_ * a_.K1;
      a.Y = labels.data_ptr<int64_t>() + s0 * B_;
      a.loss = loss_rows.data_ptr<float>() + s0 * B_;
      a.adam = adam_.data_ptr<float>() + 4 * s0;
      a.seeds = reinterpret_cast<const uint32_t*>(seeds_.data_ptr<int32_t>()) + 4 * s0;
      a.ipc.T = 0;
      if (ipc_ != nullptr) a.ipc = ipc_->begin_steps(n);
      // trace stamps: the first chunk only
      a.trace = s0 == 0 ? tr : nullptr;
      a.trace_steps = s0 == 0 ? trs : 0;
      a.tall = s0 == 0 ? ta : nullptr;
      a.tall_step = (int)trace_all_step;
      a.tall_n = s0 == 0 ? tan : 0;
      a.fault_step = (fault_step_ >= s0 && fault_step_ < s0 + n) ? (int)(fault_step_ - s0) : -1;
      const std::string why = sl::hybrid_check(a);
      TORCH_CHECK(why.empty(), "HybridEpoch: ", why);
      const hipError_t le = sl::hybrid_epoch_launch(a, st);
      TORCH_CHECK(le == hipSuccess, "hybrid epoch launch: ", hipGetErrorString(le));
    }
    ++launches_;
    if (fault_step_ >= 0) fault_step_ = -1;   // one injected fault per arming
    const int e = err_.item<int>();   // one sync per client epoch
    TORCH_CHECK(e == 0, "hybrid server epoch: an in-launch wait gave up (error word ", e,
                "; 2 = a hand-off timed out, 4 = the peer-mapped fc2 exchange failed)");
    return py::make_tuple(fwd_count + S, t + S, S * B_);
  }

  // tests: in the next run, step `step`'s first hand-off wait is never met (it times out,
  // err 2, and every other wait gives up), as a lost hand-off would; -1 disarms
  void set_fault_step(int64_t step) { fault_step_ = step; }
  int64_t max_steps() const { return max_steps_; }

  // the device table (tile runs, row-block owners / counts, column-block counts) for checks
  at::Tensor table() const { return tab_.clone(); }

 private:
  // tile runs and arrival counts (hybrid.h HyArgs.tab); "" or the reason the shape is refused
  std::string tables() {
    sl::HyArgs& a = a_;
    const int G = a.G, nrb = a.nrb, ncb = a.ncb, NC = a.NC, T = a.ntile;
    if (a.N1 % 4 || a.N1 < 4) return "fc1 shard width % 4";
    const int Q4 = a.N1 / 4;
    std::vector<int> tab(G + 1 + 2 * nrb + NC, 0);
    // balanced contiguous runs; with fewer tiles than workgroups the first T workgroups take
    // one tile each (no empty run between two workgroups that share a row block)
    for (int w = 0; w <= G; ++w) tab[w] = T >= G ? (int)((int64_t)w * T / G) : std::min(w, T);
    auto wg_of = [&](int t) {   // the workgroup whose run holds tile t
      int lo = 0, hi = G - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (tab[mid] <= t) lo = mid;
        else hi = mid - 1;
      }
      return lo;
    };
    auto colblk = [&](int n4) { return (int)(((int64_t)(n4 + 1) * NC + Q4 - 1) / Q4) - 1; };
    for (int rb = 0; rb < nrb; ++rb) {
      const int w0 = wg_of(rb * ncb), w1 = wg_of(std::min((rb + 1) * ncb, T) - 1);
      tab[G + 1 + rb] = w0;
      tab[G + 1 + nrb + rb] = w1 - w0 + 1;
      if (w1 - w0 + 1 > sl::kHySlots) return "an fc1 row block spans more workgroups than the partial slots";
      const int blo = colblk((16 * rb) / 4), bhi = colblk((std::min(16 * rb + 16, a.N1) - 1) / 4);
      for (int b = blo; b <= bhi; ++b) ++tab[G + 1 + 2 * nrb + b];
    }
    for (int w = 0; w < G; ++w) {
      if (tab[w + 1] <= tab[w]) continue;
      const int runs = (tab[w + 1] - 1) / ncb - tab[w] / ncb + 1;
      if (runs > sl::kHyRuns) return "a tile run touches more than 3 fc1 row blocks";
    }
    for (int b = 0; b < NC; ++b)
      if (tab[G + 1 + 2 * nrb + b] < 1) return "an fc2 column block without fc1 rows";
    tab_ = at::tensor(tab, at::TensorOptions().dtype(at::kInt)).to(L_[0].W.device());
    return "";
  }

  HyLayer L_[3];
  int kind_ = 2, col_off1_ = 0, B_ = 16, dev_ = 0, clock_khz_ = 100000;
  double lr_ = 0, beta1_ = 0, beta2_ = 0, eps_ = 0, wd_ = 0, mom_ = 0, p1_ = 0, p2_ = 0, timeout_s_ = 30.0;
  sl::IpcAllReduce* ipc_ = nullptr;
  sl::HyArgs a_{};
  bool ok_ = false;
  std::string why_;
  int64_t max_steps_ = 1, fault_step_ = -1, launches_ = 0;
  at::Tensor HB_, cnt_, err_, shard_n_, tab_, adam_, seeds_;
};

}  // namespace

void sl_register_hybrid(py::module& m) {
  py::class_<HybridEpoch>(m, "HybridEpoch")
      .def(py::init<const py::dict&>())
      .def("ok", &HybridEpoch::ok)
      .def("why", &HybridEpoch::why)
      .def("workgroups", &HybridEpoch::workgroups)
      .def("table", &HybridEpoch::table)
      .def("set_fault_step", &HybridEpoch::set_fault_step)
      .def("max_steps", &HybridEpoch::max_steps)
      .def("run", &HybridEpoch::run, py::arg("acts"), py::arg("labels"), py::arg("loss_rows"),
           py::arg("seed_base"), py::arg("fwd_count"), py::arg("t"), py::arg("trace") = py::none(),
           py::arg("trace_all") = py::none(), py::arg("trace_all_step") = 0, py::arg("step_rows") = py::none());
}
