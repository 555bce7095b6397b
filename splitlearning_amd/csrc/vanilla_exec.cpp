// Host side of the vanilla persistent split epoch (`_C.VanillaEpoch`, csrc/vanilla.hip).
//
// Reference: the vanilla hot loop, data_entities_vanilla.py:66-76.  One `run` call = ONE
// cooperative launch over every batch of a co-located Alice's epoch order, a short final batch
// included (its rows padded to B with ignored labels and zero activations, its CE mean over its
// real rows).  The host builds the per-step tables (batch rows, labels, CE scales, dropout
// seeds: host.h step_seed == ops/rng.py), the two fc1 tile-run tables, zeroes the counters (in
// the launch), launches and reads the kernel's error word once.
//
// Remote Alice (cfg channel / peer / G; BASELINE config 3's remote placements): `run_remote`
// is Bob's side of a remote Alice's epoch, the launch sending and receiving the per-batch
// messages on the peer-mapped channel itself (csrc/vanilla.hip REM); her side stays
// csrc/split.cpp run_alice, so the per-batch run_bob is the drop-in fallback.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <cstdlib>
#include <string>
#include <tuple>
#include <vector>

#include "host.h"
#include "ipc_p2p.h"
#include "vanilla.h"

namespace py = pybind11;

namespace {

at::Tensor va_get(const py::dict& d, const char* k) {
  TORCH_CHECK(d.contains(k) && !d[k].is_none(), "VanillaEpoch: missing '", k, "'");
  return d[k].cast<at::Tensor>();
}

void va_f32(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "VanillaEpoch: ", what, " f32 GPU");
}

class VanillaEpoch {
 public:
  // cfg: layers = [3 dicts {W, b, s0, sb0}] (Bob's model2_sisa, SGD-momentum buffers), lr /
  // momentum / wd (Bob), alice = {w [32, 1, 3, 3], b [32], s0w, s0b} + alice_lr / alice_momentum /
  // alice_wd, x (uint8 shard [N, 784]), y (int64 labels [N]), p1 / p2, B, timeout_s,
  // workgroups (0: cooperative launch of 256).  Remote Alice: channel (an open IpcChannel) and
  // peer (her rank) in place of alice / x / y; G workgroups (default 256)
  explicit VanillaEpoch(const py::dict& cfg) {
    auto layers = cfg["layers"].cast<std::vector<py::dict>>();
    TORCH_CHECK(layers.size() == 3, "VanillaEpoch drives model2_sisa's 3 layers");
    for (int i = 0; i < 3; ++i) {
      const py::dict& d = layers[i];
      W_[i] = va_get(d, "W");
      b_[i] = va_get(d, "b");
      s0_[i] = va_get(d, "s0");
      sb0_[i] = va_get(d, "sb0");
      for (const at::Tensor* t : {&W_[i], &b_[i], &s0_[i], &sb0_[i]}) va_f32(*t, "layer tensors");
      TORCH_CHECK(W_[i].dim() == 2 && s0_[i].sizes() == W_[i].sizes() && b_[i].numel() == W_[i].size(0) &&
                      sb0_[i].numel() == W_[i].size(0),
                  "layer shapes");
    }
    TORCH_CHECK(W_[1].size(1) == W_[0].size(0) && W_[2].size(1) == W_[1].size(0), "layer chain shapes");
    rem_ = cfg.contains("channel") && !cfg["channel"].is_none();
    if (rem_) {
      const py::object ch = cfg["channel"];
      TORCH_CHECK(py::isinstance<sl::IpcChannel>(ch), "VanillaEpoch: channel must be an IpcChannel");
      chan_ = ch.cast<sl::IpcChannel*>();
      channel_ = ch;   // keep the channel alive with the executor
      peer_ = cfg["peer"].cast<int>();
      TORCH_CHECK(chan_->opened() && peer_ >= 0 && peer_ < chan_->size() && peer_ != chan_->rank(),
                  "VanillaEpoch: an open channel and the Alice's rank");
    } else {
      py::dict al = cfg["alice"].cast<py::dict>();
      cw_ = va_get(al, "w");
      cb_ = va_get(al, "b");
      cmw_ = va_get(al, "s0w");
      cmb_ = va_get(al, "s0b");
      for (const at::Tensor* t : {&cw_, &cb_, &cmw_, &cmb_}) va_f32(*t, "conv tensors");
      TORCH_CHECK(cw_.numel() == 288 && cb_.numel() == 32 && cmw_.numel() == 288 && cmb_.numel() == 32,
                  "conv 32 x 1 x 3 x 3");
      x_ = va_get(cfg, "x");
      y_ = va_get(cfg, "y");
      TORCH_CHECK(x_.is_cuda() && x_.scalar_type() == at::kByte && x_.is_contiguous() && x_.numel() % 784 == 0,
                  "shard pixels uint8 [N, 784]");
      TORCH_CHECK(y_.is_cuda() && y_.scalar_type() == at::kLong && y_.numel() * 784 == x_.numel(), "labels int64 [N]");
    }
    B_ = cfg["B"].cast<int>();
    const double p1 = cfg["p1"].cast<double>(), p2 = cfg["p2"].cast<double>();
    timeout_s_ = cfg.contains("timeout_s") ? cfg["timeout_s"].cast<double>() : 30.0;

    dev_ = W_[0].device().index();
    int cus = 0;
    TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_) == hipSuccess, "CU count");
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_) != hipSuccess || khz <= 0) khz = 100000;

    sl::VaArgs& a = a_;
    a = sl::VaArgs{};
    a.N1 = (int)W_[0].size(0);
    a.K1 = (int)W_[0].size(1);
    a.N2 = (int)W_[1].size(0);
    a.C = (int)W_[2].size(0);
    a.C4 = (a.C + 3) & ~3;
    a.M = B_;
    a.G = rem_ && cfg.contains("G") ? cfg["G"].cast<int>() : sl::kVaG;
    a.rem = rem_ ? 1 : 0;
    const int wg = cfg.contains("workgroups") ? cfg["workgroups"].cast<int>() : 0;
    a.coop = wg > 0 ? 0 : 1;
    a.fault_step = -1;
    a.NC = a.G / sl::kVaNR;
    a.HW = a.N2 / 4;
    a.nrb = (a.N1 + 15) / 16;
    a.ncb = (a.K1 + 255) / 256;
    a.ntile = a.nrb * a.ncb;
    a.ignore = -100;
    a.thr1 = p1 > 0 ? (uint32_t)(p1 * 4294967296.0) : 0u;
    a.thr2 = p2 > 0 ? (uint32_t)(p2 * 4294967296.0) : 0u;
    a.dsc1 = p1 > 0 ? (float)(1.0 / (1.0 - p1)) : 1.f;
    a.dsc2 = p2 > 0 ? (float)(1.0 / (1.0 - p2)) : 1.f;
    a.o = sl::make_opt_raw(1, cfg["lr"].cast<double>(), 0, 0, 0, cfg["wd"].cast<double>(),
                           cfg["momentum"].cast<double>(), 0, nullptr);
    a.oa = rem_ ? sl::make_opt_raw(1, 0.0, 0, 0, 0, 0.0, 0.0, 0, nullptr)
                : sl::make_opt_raw(1, cfg["alice_lr"].cast<double>(), 0, 0, 0, cfg["alice_wd"].cast<double>(),
                                   cfg["alice_momentum"].cast<double>(), 0, nullptr);
    why_ = cus < a.G ? "fewer CUs than workgroups" : "";
    if (why_.empty() && rem_) {
      // placeholders the check requires; the launch's own are set per chunk
      a.Yrem = reinterpret_cast<int64_t*>(16);
      a.lk.sdata[0] = reinterpret_cast<float*>(16);
      a.lk.rdata[0] = reinterpret_cast<const float*>(16);
      if (chan_->cap() < act_words(B_)) why_ = "the channel is too small for a batch";
    }
    if (why_.empty()) why_ = sl::vanilla_check(a);
    if (why_.empty()) why_ = tables();
    if (why_.empty()) {
      auto opt = at::TensorOptions().dtype(at::kFloat).device(W_[0].device());
      int64_t off = 0;
      auto take = [&](int64_t n) {
        const int64_t o = off;
        off += (n + 3) & ~3LL;
        return (int)o;
      };
      a.oLA = take(2LL * a.nrb * sl::kVaSlots * 256);
      a.oH1 = take(2LL * 16 * a.N1);
      a.oFP = take(2LL * a.NC * 16 * a.N2);
      a.oLP = take(2LL * a.HW * 16 * a.C4);
      a.oDL = take(2LL * 16 * a.C4);
      a.oDZ = take(2LL * 16 * a.N2);
      a.oDP = take(2LL * sl::kVaNR * 16 * a.N1);
      a.oDX = take((int64_t)a.ncb * sl::kVaDxSlots * 16 * 256);
      a.oCWP = take(2LL * 32 * 8 * 16);
      HB_ = at::zeros({off}, opt);
      a.HB = HB_.data_ptr<float>();
      cnt_ = at::zeros({(int64_t)sl::kVaCounters * sl::kVaStride}, opt.dtype(at::kInt));
      err_ = at::zeros({1}, opt.dtype(at::kInt));
      std::vector<int> sn(sl::kVaSeams * 8, 0);
      for (int w = 0; w < a.G; ++w) {
        ++sn[0 * 8 + (w & 7)];                 // F: every tile
        if (w < a.HW) ++sn[1 * 8 + (w & 7)];   // L: head workgroups
        if (w < a.M) ++sn[2 * 8 + (w & 7)];    // D: softmax workgroups
        if (w < a.HW) ++sn[3 * 8 + (w & 7)];   // Z: head workgroups
        ++sn[4 * 8 + (w & 7)];                 // X: every conv job
      }
      shard_n_ = at::tensor(sn, at::TensorOptions().dtype(at::kInt)).to(W_[0].device());
      a.cnt = reinterpret_cast<unsigned*>(cnt_.data_ptr<int>());
      a.shard_n = shard_n_.data_ptr<int>();
      a.err = err_.data_ptr<int>();
      a.tab = tab_.data_ptr<int>();
      a.timeout = (int64_t)(timeout_s_ * 1000.0 * khz);
      auto setL = [&](sl::ResLayer& r, int i) {
        r.W = W_[i].data_ptr<float>();
        r.b = b_[i].data_ptr<float>();
        r.m = s0_[i].data_ptr<float>();
        r.mb = sb0_[i].data_ptr<float>();
        r.v = nullptr;
        r.vb = nullptr;
      };
      setL(a.L1, 0);
      setL(a.L2, 1);
      setL(a.L3, 2);
      if (!rem_) {
        a.img = x_.data_ptr<uint8_t>();
        a.cw = cw_.data_ptr<float>();
        a.cb = cb_.data_ptr<float>();
        a.cmw = cmw_.data_ptr<float>();
        a.cmb = cmb_.data_ptr<float>();
      }
      std::string why;
      sl::vanilla_fits(a, dev_, &why);
      why_ = why;
    }
    ok_ = why_.empty();
  }

  bool ok() const { return ok_; }
  std::string why() const { return why_; }

  // One epoch over `order` (int64 shard rows [n], on the device): ceil(n / B) steps in one
  // launch.  Per-row losses -> loss_rows [>= S * B] (padding rows 0).  t_a / t_b: optimizer
  // steps so far; fwd_count: Bob's forward counter (dropout hash).  Returns (t_a, t_b,
  // fwd_count) advanced by the step count.  Raises when an in-launch wait gave up.
  py::tuple run(const at::Tensor& order, at::Tensor& loss_rows, int64_t t_a, int64_t t_b, int64_t fwd_count,
                int64_t seed_base, const c10::optional<at::Tensor>& trace_all, int64_t trace_step) {
    TORCH_CHECK(ok_, "VanillaEpoch: ", why_);
    TORCH_CHECK(!rem_, "VanillaEpoch.run: a co-located Alice (run_remote serves a remote one)");
    TORCH_CHECK(order.is_cuda() && order.scalar_type() == at::kLong && order.dim() == 1, "order int64 [n] on the GPU");
    const int64_t n = order.numel();
    const int64_t S = (n + B_ - 1) / B_;
    if (S == 0) return py::make_tuple(t_a, t_b, fwd_count);
    const at::Device dev = order.device();
    auto lopt = at::TensorOptions().dtype(at::kLong).device(dev);
    rows_ = at::full({S * B_}, -1, lopt);
    rows_.narrow(0, 0, n).copy_(order);
    labels_ = at::full({S * B_}, -100, lopt);
    labels_.narrow(0, 0, n).copy_(y_.index_select(0, order));
    epoch(n, S, loss_rows, fwd_count, seed_base, trace_all, trace_step, dev);
    return py::make_tuple(t_a + S, t_b + S, fwd_count + S);
  }

  // Bob's side of a remote Alice's epoch of n samples (her side: csrc/split.cpp run_alice):
  // the per-batch messages -- her activation + labels in, the cut gradient out -- go over the
  // channel from inside the launch, in run_bob's order and sizes.  Returns (t_b, fwd_count)
  // advanced by the step count.  Raises when an in-launch wait gave up (fail-stop: she is
  // then stopped at a message of this epoch and times out on her side).
  py::tuple run_remote(int64_t n, at::Tensor& loss_rows, int64_t t_b, int64_t fwd_count, int64_t seed_base,
                       const c10::optional<at::Tensor>& trace_all, int64_t trace_step) {
    TORCH_CHECK(ok_, "VanillaEpoch: ", why_);
    TORCH_CHECK(rem_, "VanillaEpoch.run_remote: configured with a channel and peer");
    const int64_t S = n > 0 ? (n + B_ - 1) / B_ : 0;
    if (S == 0) return py::make_tuple(t_b, fwd_count);
    epoch(n, S, loss_rows, fwd_count, seed_base, trace_all, trace_step, W_[0].device());
    return py::make_tuple(t_b + S, fwd_count + S);
  }

  // (op, peer, bytes) of every message the last run_remote issued, in issue order (run_bob's)
  std::vector<std::tuple<std::string, int, int64_t>> messages() const { return log_; }

  void set_fault_step(int64_t s) { fault_step_ = (int)s; }
  bool remote() const { return rem_; }
  int workgroups() const { return a_.G; }
  void set_max_steps(int64_t s) { max_steps_ = std::max<int64_t>(1, std::min<int64_t>(s, sl::kVaMaxS)); }
  at::Tensor table() const { return tab_.clone(); }

 private:
  // the vanilla activation message's words: split.cpp act_msg_words (M x 5408 activation, then
  // M int64 labels, padded to 16 bytes)
  static int64_t act_words(int M) { return ((int64_t)M * 5408 + 2 * (int64_t)M + 3) / 4 * 4; }

  // One epoch of S steps over n samples as launches of at most max_steps_ steps: the per-step
  // tables (rows, CE scale, dropout seeds), then per chunk (remote: its run of channel messages)
  // one launch; one read of the error word per chunk.
  void epoch(int64_t n, int64_t S, at::Tensor& loss_rows, int64_t fwd_count, int64_t seed_base,
             const c10::optional<at::Tensor>& trace_all, int64_t trace_step, const at::Device& dev) {
    TORCH_CHECK(loss_rows.is_cuda() && loss_rows.scalar_type() == at::kFloat && loss_rows.numel() >= S * B_,
                "loss_rows f32 [>= S * B]");
    std::vector<float> tabf(4 * S, 0.f);
    std::vector<int32_t> seeds(4 * S);
    auto rows_at = [&](int64_t i) { return (int)std::min<int64_t>(B_, n - i * B_); };
    for (int64_t i = 0; i < S; ++i) {
      const int64_t rows = rows_at(i);
      tabf[4 * i] = (float)rows;
      tabf[4 * i + 2] = (float)(1.0 / (double)rows);
      const uint64_t s0 = sl::step_seed((uint64_t)seed_base, 0, (uint64_t)(fwd_count + 1 + i));
      const uint64_t s1 = sl::step_seed((uint64_t)seed_base, 1, (uint64_t)(fwd_count + 1 + i));
      seeds[4 * i] = (int32_t)(uint32_t)(s0 & 0xffffffffull);
      seeds[4 * i + 1] = (int32_t)(uint32_t)(s0 >> 32);
      seeds[4 * i + 2] = (int32_t)(uint32_t)(s1 & 0xffffffffull);
      seeds[4 * i + 3] = (int32_t)(uint32_t)(s1 >> 32);
    }
    tabf_ = at::from_blob(tabf.data(), {4 * S}, at::TensorOptions().dtype(at::kFloat)).to(dev);
    seeds_ = at::from_blob(seeds.data(), {4 * S}, at::TensorOptions().dtype(at::kInt)).to(dev);
    const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    TORCH_CHECK(hipMemsetAsync(a_.err, 0, sizeof(int), st) == hipSuccess, "vanilla error word");
    // launches of at most kVaMaxS steps (one launch of S steps is bitwise S one-step launches)
    const int64_t cs = std::min<int64_t>(S, max_steps_);
    xr_ = at::empty({cs * 16 * a_.K1}, at::TensorOptions().dtype(at::kFloat).device(dev));
    if (rem_) yrem_ = at::empty({cs * B_}, at::TensorOptions().dtype(at::kLong).device(dev));
    log_.clear();
    for (int64_t s0 = 0; s0 < S; s0 += cs) {
      // a chunk whose wait gave up stops the epoch here (host check between chunks, as HybridEpoch)
      if (s0 > 0 && err_.item<int>() != 0) break;
      const int64_t ns = std::min(cs, S - s0);
      sl::VaArgs a = a_;
      a.S = (int)ns;
      a.Xr = xr_.data_ptr<float>();
      a.loss = loss_rows.data_ptr<float>() + s0 * B_;
      a.adam = tabf_.data_ptr<float>() + 4 * s0;
      a.seeds = reinterpret_cast<const uint32_t*>(seeds_.data_ptr<int32_t>()) + 4 * s0;
      if (rem_) {
        std::vector<int64_t> sends, recvs;
        for (int64_t i = s0; i < s0 + ns; ++i) {
          recvs.push_back(act_words(rows_at(i)));
          sends.push_back((int64_t)rows_at(i) * a_.K1);
          log_.emplace_back("recv", peer_, recvs.back() * 4);
          log_.emplace_back("send", peer_, sends.back() * 4);
        }
        const sl::P2PRun r = chan_->run(peer_, st, sends, recvs);
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
        a.Yrem = yrem_.data_ptr<int64_t>();
        a.rows = nullptr;
        a.Y = nullptr;
      } else {
        a.rows = rows_.data_ptr<int64_t>() + s0 * B_;
        a.Y = labels_.data_ptr<int64_t>() + s0 * B_;
      }
      if (trace_all.has_value() && s0 == 0) {
        TORCH_CHECK(trace_all->is_cuda() && trace_all->scalar_type() == at::kLong && trace_all->is_contiguous() &&
                        trace_all->numel() % (16LL * a_.G) == 0,
                    "trace_all int64 [steps, G, 16]");
        a.tall = trace_all->data_ptr<int64_t>();
        a.tall_n = (int)(trace_all->numel() / (16LL * a_.G));
        a.tall_step = (int)(trace_step - s0);
      }
      a.fault_step = fault_step_ >= s0 && fault_step_ < s0 + ns ? (int)(fault_step_ - s0) : -1;
      const hipError_t le = sl::vanilla_epoch_launch(a, st);
      TORCH_CHECK(le == hipSuccess, "vanilla epoch launch: ", hipGetErrorString(le));
    }
    fault_step_ = -1;
    const int e = err_.item<int>();
    TORCH_CHECK(e == 0, "vanilla split epoch: an in-launch wait gave up (error word ", e, ")");
  }

  // forward (row-major, hybrid_exec.cpp's) and update (column-major) tile runs
  std::string tables() {
    sl::VaArgs& a = a_;
    const int G = a.G, nrb = a.nrb, ncb = a.ncb, NC = a.NC, T = a.ntile;
    const int Q4 = a.N1 / 4;
    if (T < G) return "fewer fc1 tiles than workgroups";
    std::vector<int> tab(G + 1 + 2 * nrb + NC, 0);
    for (int w = 0; w <= G; ++w) tab[w] = (int)((int64_t)w * T / G);
    auto wg_of = [&](const std::vector<int>& t0, int base, int t) {
      int lo = 0, hi = G - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (t0[base + mid] <= t) lo = mid;
        else hi = mid - 1;
      }
      return lo;
    };
    auto colblk = [&](int n4) { return (int)(((int64_t)(n4 + 1) * NC + Q4 - 1) / Q4) - 1; };
    for (int rb = 0; rb < nrb; ++rb) {
      const int w0 = wg_of(tab, 0, rb * ncb), w1 = wg_of(tab, 0, std::min((rb + 1) * ncb, T) - 1);
      tab[G + 1 + rb] = w0;
      tab[G + 1 + nrb + rb] = w1 - w0 + 1;
      if (w1 - w0 + 1 > sl::kVaSlots) return "an fc1 row block spans more workgroups than the forward slots";
      const int blo = colblk((16 * rb) / 4), bhi = colblk((std::min(16 * rb + 16, a.N1) - 1) / 4);
      for (int b = blo; b <= bhi; ++b) ++tab[G + 1 + 2 * nrb + b];
    }
    for (int w = 0; w < G; ++w) {
      if (tab[w + 1] <= tab[w]) continue;
      const int runs = (tab[w + 1] - 1) / ncb - tab[w] / ncb + 1;
      if (runs > sl::kVaRuns) return "a forward run touches more than 3 fc1 row blocks";
    }
    for (int b = 0; b < NC; ++b)
      if (tab[G + 1 + 2 * nrb + b] < 1) return "an fc2 column block without fc1 rows";
    // update runs: G balanced column-major runs over all tiles (tile v: column block v / nrb, row
    // block v % nrb), as before, but dealt to the workgroups by the row band their first tile
    // falls in -- run k goes to a workgroup of XCD x (w % 8 == x under round-robin dispatch)
    // when its first row block is in band x of 8 -- so the runs of one XCD stage the dz1 of
    // ~1/4 of the row blocks instead of all of them (the staging is an L2 <- fabric fetch).
    // Each run keeps its slot among the workgroups touching its column blocks.
    a.oU = (int)tab.size();
    tab.resize(a.oU + ncb, 0);
    a.oUW = (int)tab.size();
    tab.resize(a.oUW + 4 * G, 0);
    a.oUS = (int)tab.size();
    std::vector<int> run_of(G, -1);
    // SL_VA_XCD_RUNS=0: runs dealt in order (A/B)
    const char* env_x = std::getenv("SL_VA_XCD_RUNS");
    const bool xcd_runs = !(env_x && env_x[0] == '0');
    if (G % 8 == 0 && nrb >= 64 && xcd_runs) {
      std::vector<int> used(G, 0), spill;
      std::vector<int> next(8, 0);
      for (int k = 0; k < G; ++k) {
        const int v0 = (int)((int64_t)k * T / G);
        const int x = (int)((int64_t)(v0 % nrb) * 8 / nrb);
        if (next[x] < G / 8) {
          const int w = x + 8 * next[x]++;
          run_of[w] = k;
          used[w] = 1;
        } else {
          spill.push_back(k);
        }
      }
      size_t q = 0;
      for (int w = 0; w < G && q < spill.size(); ++w)
        if (!used[w]) run_of[w] = spill[q++];
    } else {
      for (int w = 0; w < G; ++w) run_of[w] = w;
    }
    auto fill = [&]() -> std::string {
      tab.resize(a.oUS);
      tab.resize(a.oUS + (size_t)G * ncb, -1);
      std::vector<int> cnt(ncb, 0);
      for (int k = 0; k < G; ++k) {
        // slots per column block in run order (the sum order of the cut-gradient partials)
        int w = -1;
        for (int x = 0; x < G; ++x)
          if (run_of[x] == k) { w = x; break; }
        if (w < 0) return "update run table";
        const int v0 = (int)((int64_t)k * T / G), v1 = (int)((int64_t)(k + 1) * T / G);
        if (v1 - v0 > sl::kVaMaxRun) return "an update run longer than 28 tiles";
        tab[a.oUW + 4 * w] = v0;
        tab[a.oUW + 4 * w + 1] = v1;
        tab[a.oUW + 4 * w + 2] = 0;
        tab[a.oUW + 4 * w + 3] = nrb;
        if (v1 <= v0) continue;
        for (int cb = v0 / nrb; cb <= (v1 - 1) / nrb; ++cb) {
          tab[a.oUS + (size_t)w * ncb + cb] = cnt[cb]++;
          if (cnt[cb] > sl::kVaDxSlots) return "an fc1 column block spans more workgroups than the dx slots";
        }
      }
      for (int cb = 0; cb < ncb; ++cb) tab[a.oU + cb] = cnt[cb];
      return "";
    };
    {
      const std::string e = fill();
      if (!e.empty()) return e;
    }
    tab_ = at::tensor(tab, at::TensorOptions().dtype(at::kInt)).to(W_[0].device());
    return "";
  }

  at::Tensor W_[3], b_[3], s0_[3], sb0_[3];
  at::Tensor cw_, cb_, cmw_, cmb_, x_, y_;
  int B_ = 16, dev_ = 0, fault_step_ = -1;
  int64_t max_steps_ = sl::kVaMaxS;
  double timeout_s_ = 30.0;
  sl::VaArgs a_{};
  bool ok_ = false;
  std::string why_;
  at::Tensor HB_, cnt_, err_, shard_n_, tab_, tabf_, seeds_, rows_, labels_, xr_, yrem_;
  bool rem_ = false;
  sl::IpcChannel* chan_ = nullptr;
  py::object channel_;
  int peer_ = -1;
  std::vector<std::tuple<std::string, int, int64_t>> log_;
};

}  // namespace

void sl_register_vanilla(py::module& m) {
  py::class_<VanillaEpoch>(m, "VanillaEpoch")
      .def(py::init<const py::dict&>())
      .def("ok", &VanillaEpoch::ok)
      .def("why", &VanillaEpoch::why)
      .def("table", &VanillaEpoch::table)
      .def("set_fault_step", &VanillaEpoch::set_fault_step)
      .def("set_max_steps", &VanillaEpoch::set_max_steps)
      .def("run", &VanillaEpoch::run, py::arg("order"), py::arg("loss_rows"), py::arg("t_a"), py::arg("t_b"),
           py::arg("fwd_count"), py::arg("seed_base"), py::arg("trace_all") = py::none(), py::arg("trace_step") = 0)
      .def("run_remote", &VanillaEpoch::run_remote, py::arg("n"), py::arg("loss_rows"), py::arg("t_b"),
           py::arg("fwd_count"), py::arg("seed_base"), py::arg("trace_all") = py::none(), py::arg("trace_step") = 0)
      .def("messages", &VanillaEpoch::messages)
      .def("remote", &VanillaEpoch::remote)
      .def("workgroups", &VanillaEpoch::workgroups);
}
