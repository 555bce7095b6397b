// Native executor of Bob's SISA server epoch (`_C.ServerEpoch`).
//
// Reference: bob.train_and_backward's inner loop (data_entities_vanilla_sisa.py:298-313):
// per cached batch `zero_grad; CE(model2_sisa(act), y).backward(); Adam.step()`.
// The Python engine issues each step as ~8 launches (TailEngine.train_fwd_bwd3 +
// fused_step) plus, tensor-parallel, one RCCL all-reduce; at a TP = 8 shard the GPU
// finishes a step in ~55 us and Python's issue cost is of the same order, so every
// rank's host jitter lands on the all-reduce.  This executor issues the same launch
// sequence for a whole epoch from C++:
//
//   [fc1 epilogue of the look-ahead slabs | fc1 forward]  -> h1
//   fc2 forward (split-K slabs; row-parallel: this shard's product, all-reduced by the
//     peer-mapped all-reduce fused into head_fwd (ipc_ar.h), or by RCCL before the head)
//   head_fwd + head_bwd  (fc2 epilogue, fc3, softmax-CE, fc3 dgrad, fc2 ReLU/dropout bwd)
//   fc2 dgrad (+ fc1 ReLU/dropout mask)                     -> dz1
//   wgrad_group: fc1/fc2/fc3 dW fused into Adam/SGD, plus fc1's product for the next
//   full batch with the updated weights (look-ahead)
//
// Same kernels, arguments, dropout seeds (host.h step_seed == ops/rng.py) and Adam step
// counts as the Python path, so results are bit-identical to it
// (tests/test_graphs_gpu.py::test_native_server_epoch_matches_python).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <string>

#include "comm.h"
#include "common.h"
#include "fused.h"
#include "host.h"

namespace sl {
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

void ck(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e)); }

at::Tensor get(const py::dict& d, const char* k) {
  TORCH_CHECK(d.contains(k), "ServerEpoch: missing '", k, "'");
  return d[k].cast<at::Tensor>();
}

struct Layer {
  at::Tensor W, b, s0, s1, sb0, sb1;   // s1 / sb1 undefined for SGD
  int N = 0, K = 0;
};

class ServerEpoch {
 public:
  // cfg: layers = [3 dicts {W, b, s0, s1, sb0, sb1}], kind/lr/beta1/beta2/eps/wd/momentum,
  // p1, p2 (dropout), col_off1, row2 (fc2 row-parallel), comm (TpComm | None),
  // workspaces: pn, p2ws, fwdws, dgws, headws, h1, h2, dz1, dz2, dlog (each for B rows).
  explicit ServerEpoch(const py::dict& cfg) {
    auto layers = cfg["layers"].cast<std::vector<py::dict>>();
    TORCH_CHECK(layers.size() == 3, "ServerEpoch drives the 3-layer server tail");
    for (int i = 0; i < 3; ++i) {
      Layer& L = L_[i];
      const py::dict& d = layers[i];
      L.W = get(d, "W");
      L.b = get(d, "b");
      L.s0 = get(d, "s0");
      L.sb0 = get(d, "sb0");
      if (d.contains("s1") && !d["s1"].is_none()) L.s1 = get(d, "s1");
      if (d.contains("sb1") && !d["sb1"].is_none()) L.sb1 = get(d, "sb1");
      for (const at::Tensor* t : {&L.W, &L.b, &L.s0, &L.sb0}) {
        TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), "layer tensors: f32 GPU");
      }
      TORCH_CHECK(L.W.dim() == 2 && L.W.size(1) % 4 == 0, "W [N, K] with K % 4 == 0");
      L.N = (int)L.W.size(0);
      L.K = (int)L.W.size(1);
      TORCH_CHECK(L.b.numel() == L.N && L.s0.sizes() == L.W.sizes() && L.sb0.numel() == L.N, "layer state shapes");
    }
    TORCH_CHECK(L_[1].K == L_[0].N && L_[2].K == L_[1].N, "layer chain shapes");
    TORCH_CHECK(L_[1].N % 4 == 0, "fc2 width % 4");
    kind_ = cfg["kind"].cast<int>();
    TORCH_CHECK(kind_ == 1 || kind_ == 2, "SGD-momentum or Adam");
    if (kind_ == 2)
      for (auto& L : L_) TORCH_CHECK(L.s1.defined() && L.sb1.defined() && L.s1.sizes() == L.W.sizes(), "Adam v");
    lr_ = cfg["lr"].cast<double>();
    beta1_ = cfg["beta1"].cast<double>();
    beta2_ = cfg["beta2"].cast<double>();
    eps_ = cfg["eps"].cast<double>();
    wd_ = cfg["wd"].cast<double>();
    mom_ = cfg["momentum"].cast<double>();
    p1_ = cfg["p1"].cast<double>();
    p2_ = cfg["p2"].cast<double>();
    col_off1_ = cfg["col_off1"].cast<int>();
    row2_ = cfg["row2"].cast<bool>();
    if (!cfg["comm"].is_none()) comm_ = cfg["comm"].cast<sl::TpComm*>();
    // a peer-mapped all-reduce without an RCCL communicator (ranks that share a GPU, where
    // RCCL refuses the pair: tests/test_tp_processes_gpu.py)
    if (comm_ == nullptr && cfg.contains("ipc") && !cfg["ipc"].is_none()) ipc_ = cfg["ipc"].cast<sl::IpcAllReduce*>();
    // emulate_tp: a shard executor of a single-process tensor-parallel emulation
    // (tp_emulate_epoch does the all-reduce); otherwise a row-parallel fc2 needs RCCL
    emulate_ = cfg.contains("emulate_tp") && cfg["emulate_tp"].cast<bool>();
    TORCH_CHECK(!row2_ || comm_ != nullptr || ipc_ != nullptr || emulate_,
                "a row-parallel fc2 needs the native communicator");
    // grouped cross-entropy (SISA-concat's k heads, protocols/concat.py): labels [n, G], per-
    // (row, group) loss scales [n, G] passed to run(), losses [n, G]
    G_ = cfg.contains("groups") ? cfg["groups"].cast<int>() : 1;
    TORCH_CHECK(G_ >= 1 && L_[2].N % G_ == 0, "fc3 width % groups");
    B_ = cfg["B"].cast<int>();
    TORCH_CHECK(B_ >= 1 && B_ <= 64, "batch 1..64 (look-ahead row chunks of the wgrad kernel)");
    pn_ = get(cfg, "pn");
    p2ws_ = get(cfg, "p2ws");
    fwdws_ = get(cfg, "fwdws");
    dgws_ = get(cfg, "dgws");
    headws_ = get(cfg, "headws");
    h1_ = get(cfg, "h1");
    h2_ = get(cfg, "h2");
    dz1_ = get(cfg, "dz1");
    dz2_ = get(cfg, "dz2");
    dlog_ = get(cfg, "dlog");
    const int64_t S1 = (L_[0].K + 255) / 256;
    TORCH_CHECK(pn_.numel() >= S1 * B_ * L_[0].N, "pn workspace");
    TORCH_CHECK(h1_.numel() >= (int64_t)B_ * L_[0].N && dz1_.numel() >= (int64_t)B_ * L_[0].N, "h1 / dz1");
    TORCH_CHECK(h2_.numel() >= (int64_t)B_ * L_[1].N && dz2_.numel() >= (int64_t)B_ * L_[1].N, "h2 / dz2");
    TORCH_CHECK(dlog_.numel() >= (int64_t)B_ * L_[2].N, "dlog");
    TORCH_CHECK(p2ws_.numel() >= (int64_t)16 * B_ * L_[1].N, "fc2 slab workspace");
    TORCH_CHECK(headws_.numel() >= (int64_t)sl::head3_slices(L_[1].N) * B_ * L_[2].N, "head workspace");
  }

  // One epoch over acts [n, K1] / labels [n] in batches of B.  `pre`: fc1's product for the
  // first batch is pending in pn (look-ahead prologue / previous step).  Returns the
  // updated (fwd_count, t, pre).
  py::tuple run(const at::Tensor& acts, const at::Tensor& labels, at::Tensor& loss_rows, int64_t seed_base,
                int64_t fwd_count, int64_t t, bool pre, bool lookahead, const c10::optional<at::Tensor>& gscale) {
    TORCH_CHECK(!emulate_, "an emulate_tp shard executor is driven by tp_emulate_epoch, not run()");
    check_batch(acts, labels, loss_rows);
    gscale_ = nullptr;
    if (G_ > 1) {
      TORCH_CHECK(gscale.has_value() && gscale->is_cuda() && gscale->scalar_type() == at::kFloat &&
                      gscale->is_contiguous() && gscale->numel() == acts.size(0) * G_,
                  "grouped CE: gscale f32 [n, groups]");
      gscale_ = gscale->data_ptr<float>();
    }
    const int64_t n = acts.size(0);
    const sl::IpcAllReduce* ipc = row2_ ? ipc_obj() : nullptr;
    for (int64_t s = 0, i = 0; s < n; s += B_, ++i) {
      // a peer-mapped wait that timed out (stalled / dead peer) raises the error word and
      // every later wait gives up at once; its host-pinned mirror is read here without a
      // device sync, so the epoch aborts within one timeout plus <= 64 queued steps
      if (ipc != nullptr && (i & 63) == 63 && ipc->host_error() != 0)
        TORCH_CHECK(false, "peer-mapped TP all-reduce: a flag wait timed out on this rank (a peer stalled or "
                           "died); aborting the server epoch at step ", i);
      Step st = begin(acts, labels, s, seed_base, fwd_count, t, pre, lookahead);
      forward_product(st);
      if (row2_ && !ipc_head(st.M)) allreduce(p2ws_.data_ptr<float>(), (size_t)st.M * L_[1].N);
      finish(st, loss_rows);
      fwd_count = st.fwd_count;
      t = st.t;
      pre = st.next_pre;
    }
    return py::make_tuple(fwd_count, t, pre);
  }

  // ---- step phases (public so a single-process tensor-parallel emulation can interleave
  // T shard executors around its own all-reduce: tp_emulate_epoch below)
  struct Step {
    int64_t s = 0;
    int M = 0;
    int64_t fwd_count = 0, t = 0;
    bool pre = false, next_pre = false, lookahead = true;
    const at::Tensor* acts = nullptr;
    const at::Tensor* labels = nullptr;
    uint64_t sd0 = 0, sd1 = 0;
  };

  void check_batch(const at::Tensor& acts, const at::Tensor& labels, const at::Tensor& loss_rows) const {
    TORCH_CHECK(acts.is_cuda() && acts.scalar_type() == at::kFloat && acts.dim() == 2 && acts.is_contiguous() &&
                    acts.size(1) == L_[0].K,
                "acts [n, K1] contiguous f32");
    const int64_t n = acts.size(0);
    TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                    labels.numel() == n * G_,
                "labels int64 [n, groups]");
    TORCH_CHECK(loss_rows.is_cuda() && loss_rows.scalar_type() == at::kFloat && loss_rows.numel() >= n * G_,
                "loss [n, groups]");
  }

  Step begin(const at::Tensor& acts, const at::Tensor& labels, int64_t s, int64_t seed_base, int64_t fwd_count,
             int64_t t, bool pre, bool lookahead) const {
    Step st;
    st.s = s;
    st.M = (int)std::min<int64_t>(B_, acts.size(0) - s);
    st.fwd_count = fwd_count + 1;
    st.t = t;
    st.pre = pre;
    st.lookahead = lookahead;
    st.acts = &acts;
    st.labels = &labels;
    st.sd0 = sl::step_seed((uint64_t)seed_base, 0, (uint64_t)st.fwd_count);
    st.sd1 = sl::step_seed((uint64_t)seed_base, 1, (uint64_t)st.fwd_count);
    return st;
  }

  // fc1 -> h1 (epilogue of the pending look-ahead slabs, or a plain forward), then fc2's
  // product into p2ws: split-K slabs, or (row-parallel fc2) this shard's unsplit partial sum
  // that the caller all-reduces before finish()
  void forward_product(Step& st) {
    const int M = st.M;
    const int K1 = L_[0].K, N1 = L_[0].N, N2 = L_[1].N;
    const int64_t S1 = (K1 + 255) / 256;
    const hipStream_t sm = stream();
    const float* x = st.acts->data_ptr<float>() + st.s * K1;
    float* h1 = h1_.data_ptr<float>();
    float* P2 = p2ws_.data_ptr<float>();
    const Epi e1 = sl::make_epi_raw(L_[0].b.data_ptr<float>(), true, p1_, st.sd0, col_off1_, nullptr);
    if (st.pre)
      ck(sl::linear_epilogue(pn_.data_ptr<float>(), N1, h1, N1, M, N1, e1, (int)S1, (int64_t)M * N1, sm),
         "fc1 epilogue");
    else
      ck(sl::linear_fwd(x, K1, L_[0].W.data_ptr<float>(), K1, h1, N1, M, N1, K1, e1, fwdws_.data_ptr<float>(),
                        fwdws_.numel(), sm),
         "fc1 forward");
    S2_ = 1;
    if (row2_ && !(ipc_head(M) || emulate_) && N1 > 1280) {
      // row-parallel fc2 all-reduced by RCCL on a wide shard: one plain product
      Epi plain{};
      plain.dscale = 1.f;
      ck(sl::linear_fwd(h1, N1, L_[1].W.data_ptr<float>(), N1, P2, N2, M, N2, N1, plain, fwdws_.data_ptr<float>(),
                        fwdws_.numel(), sm),
         "fc2 forward");
      return;
    }
    // split-K slabs, reduced by the head (single shard, the fused peer-mapped all-reduce, or the
    // single-process emulation, which sums each shard's slabs then the shards), or one unsplit
    // partial on a narrow RCCL-reduced shard (nothing to reduce before the collective)
    const int max_split = (row2_ && !(ipc_head(M) || emulate_)) ? 1 : 16;
    ck(sl::linear_fwd_partial(h1, N1, L_[1].W.data_ptr<float>(), N1, M, N2, N1, P2, p2ws_.numel(), max_split, &S2_,
                              sm),
       "fc2 forward");
  }

  // head (h2, dlogits, dz2, loss), fc1's dZ, and the grouped wgrad + optimizer step with the
  // next full batch's fc1 look-ahead
  void finish(Step& st, at::Tensor& loss_rows) {
    const int M = st.M;
    const int K1 = L_[0].K, N1 = L_[0].N, N2 = L_[1].N, C = L_[2].N;
    const hipStream_t sm = stream();
    const int64_t n = st.acts->size(0);
    const float* X = st.acts->data_ptr<float>();
    const float* x = X + st.s * K1;
    float* h1 = h1_.data_ptr<float>();
    float* h2 = h2_.data_ptr<float>();
    float* dz1 = dz1_.data_ptr<float>();
    float* dz2 = dz2_.data_ptr<float>();
    float* dlog = dlog_.data_ptr<float>();
    (void)n;
    (void)X;
    (void)x;
    (void)K1;
    const double s1 = p1_ > 0 ? 1.0 / (1.0 - p1_) : 1.0;
    const Epi e2 = sl::make_epi_raw(L_[1].b.data_ptr<float>(), true, p2_, st.sd1, 0, nullptr);
    // tensor-parallel fc2 with a peer-mapped all-reduce: head_fwd performs it (run() issued
    // no separate all-reduce for this step)
    sl::IpcStep step;
    const sl::IpcStep* ip = nullptr;
    if (row2_ && ipc_head(M)) {
      step = ipc_obj()->begin_step();
      ip = &step;
    }
    ck(sl::server_head3(p2ws_.data_ptr<float>(), S2_, (int64_t)M * N2, e2, L_[2].W.data_ptr<float>(), N2,
                        L_[2].b.data_ptr<float>(), st.labels->data_ptr<int64_t>() + st.s * G_, -100,
                        G_ > 1 ? 1.f : (float)(1.0 / M), h2, dlog, dz2, loss_rows.data_ptr<float>() + st.s * G_,
                        headws_.data_ptr<float>(), headws_.numel(), M, N2, C, sm, ip, G_,
                        gscale_ != nullptr ? gscale_ + st.s * G_ : nullptr),
       "server head");
    ck(sl::linear_dgrad(dz2, N2, L_[1].W.data_ptr<float>(), N1, h1, N1, (float)s1, dz1, N1, dgws_.data_ptr<float>(),
                        dgws_.numel(), M, N2, N1, sm),
       "fc2 dgrad");
    wgrad(st);
  }

  // the grouped wgrad + optimizer step with the next full batch's fc1 look-ahead
  void wgrad(Step& st) {
    const int M = st.M;
    const int K1 = L_[0].K, N1 = L_[0].N, N2 = L_[1].N, C = L_[2].N;
    const hipStream_t sm = stream();
    const int64_t n = st.acts->size(0);
    const float* X = st.acts->data_ptr<float>();
    const float* x = X + st.s * K1;
    float* h1 = h1_.data_ptr<float>();
    float* h2 = h2_.data_ptr<float>();
    float* dz1 = dz1_.data_ptr<float>();
    float* dz2 = dz2_.data_ptr<float>();
    float* dlog = dlog_.data_ptr<float>();
    ++st.t;
    sl::WgGroup g{};
    g.n = 3;
    const float* dzs[3] = {dz1, dz2, dlog};
    const float* As[3] = {x, h1, h2};
    const int lds[3] = {N1, N2, C}, ldas[3] = {K1, N1, N2};
    for (int i = 0; i < 3; ++i) {
      sl::WgDesc& d = g.d[i];
      Layer& L = L_[i];
      d.dz = dzs[i];
      d.ldz = lds[i];
      d.A = As[i];
      d.lda = ldas[i];
      d.W = L.W.data_ptr<float>();
      d.ldw = L.K;
      d.s0 = L.s0.data_ptr<float>();
      d.s1 = L.s1.defined() ? L.s1.data_ptr<float>() : nullptr;
      d.bias = L.b.data_ptr<float>();
      d.sb0 = L.sb0.data_ptr<float>();
      d.sb1 = L.sb1.defined() ? L.sb1.data_ptr<float>() : nullptr;
      d.N = L.N;
      d.K = L.K;
    }
    const bool next_full = st.lookahead && st.s + 2LL * B_ <= n;
    if (next_full) {
      g.xn = X + (st.s + B_) * K1;
      g.ldxn = K1;
      g.mn = B_;
      g.pn = pn_.data_ptr<float>();
    }
    const SlOpt o = sl::make_opt_raw(kind_, lr_, beta1_, beta2_, eps_, wd_, mom_, st.t, nullptr);
    ck(sl::wgrad_group(g, M, o, sm), "wgrad_group");
    st.next_pre = next_full;
  }

  // the peer-mapped all-reduce in use for this executor (attached to the RCCL communicator
  // or given bare), or null
  sl::IpcAllReduce* ipc_obj() const { return comm_ != nullptr ? comm_->ipc() : ipc_; }
  // whether step rows M run the all-reduce inside head_fwd (a stream being captured: RCCL, see
  // TpComm::allreduce_sum_f32; a message the peer-mapped region cannot hold: the separate path)
  bool ipc_head(int M) const {
    const sl::IpcAllReduce* a = ipc_obj();
    if (a == nullptr) return false;
    if ((int64_t)M * L_[1].N > a->cap() || (int64_t)M * sl::head3_slices(L_[1].N) > sl::kIpcFlags) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(stream(), &cs) == hipSuccess && cs == hipStreamCaptureStatusNone;
  }

  void allreduce(float* p, size_t n) {
    if (comm_ != nullptr)
      comm_->allreduce_sum_f32(p, n, stream());   // the attached peer-mapped path or RCCL
    else if (ipc_ != nullptr)
      ipc_->allreduce_sum_f32(p, n, stream());
    else
      TORCH_CHECK(false, "ServerEpoch: a row-parallel fc2 without a communicator");
  }

  at::Tensor product_view(int M) const { return p2ws_.narrow(0, 0, (int64_t)M * L_[1].N); }
  // this shard's fc2 product: its split-K slabs summed in slab order (as the fused head does)
  at::Tensor local_product(int M) const {
    const int64_t sl = (int64_t)M * L_[1].N;
    at::Tensor acc = p2ws_.narrow(0, 0, sl).clone();
    for (int s = 1; s < S2_; ++s) acc.add_(p2ws_.narrow(0, (int64_t)s * sl, sl));
    return acc;
  }
  // after the emulated all-reduce: the product is one reduced slab
  void set_reduced(const at::Tensor& sum, int M) {
    product_view(M).copy_(sum);
    S2_ = 1;
  }
  bool row_parallel() const { return row2_; }
  int batch() const { return B_; }

 private:
  Layer L_[3];
  int kind_ = 2;
  double lr_ = 0, beta1_ = 0, beta2_ = 0, eps_ = 0, wd_ = 0, mom_ = 0, p1_ = 0, p2_ = 0;
  int col_off1_ = 0;
  bool row2_ = false;
  sl::TpComm* comm_ = nullptr;
  sl::IpcAllReduce* ipc_ = nullptr;
  int B_ = 16;
  bool emulate_ = false;
  int S2_ = 1;
  int G_ = 1;
  const float* gscale_ = nullptr;
  at::Tensor pn_, p2ws_, fwdws_, dgws_, headws_, h1_, h2_, dz1_, dz2_, dlog_;
  static hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
};

// Single-process emulation of the tensor-parallel server epoch: T shard executors (each
// built with emulate_tp over its own shard, optimizer state and workspaces) are stepped in
// lock step on one GPU, and the row-parallel fc2's all-reduce is a sum of the T partial
// products (fixed order) copied back into every shard.  Every other launch is exactly the
// production path (ServerEpoch::run), so the shard math of the native executor is checked
// against the single-shard run without a multi-GPU box.
py::tuple tp_emulate_epoch(py::list exs, const at::Tensor& acts, const at::Tensor& labels, py::list loss_rows,
                           int64_t seed_base, int64_t fwd_count, int64_t t, bool pre, bool lookahead) {
  std::vector<ServerEpoch*> E;
  std::vector<at::Tensor> losses;
  for (auto h : exs) E.push_back(h.cast<ServerEpoch*>());
  for (auto h : loss_rows) losses.push_back(h.cast<at::Tensor>());
  TORCH_CHECK(!E.empty() && E.size() == losses.size(), "one loss buffer per shard executor");
  const int B = E[0]->batch();
  for (size_t i = 0; i < E.size(); ++i) {
    TORCH_CHECK(E[i]->batch() == B, "shard executors differ in batch size");
    E[i]->check_batch(acts, labels, losses[i]);
  }
  const bool row = E[0]->row_parallel();
  const int64_t n = acts.size(0);
  for (int64_t s = 0; s < n; s += B) {
    std::vector<ServerEpoch::Step> st;
    for (auto* e : E) st.push_back(e->begin(acts, labels, s, seed_base, fwd_count, t, pre, lookahead));
    for (size_t i = 0; i < E.size(); ++i) E[i]->forward_product(st[i]);
    if (row && E.size() > 1) {
      const int M = st[0].M;
      at::Tensor sum = E[0]->local_product(M);
      for (size_t i = 1; i < E.size(); ++i) sum.add_(E[i]->local_product(M));
      for (auto* e : E) e->set_reduced(sum, M);
    }
    for (size_t i = 0; i < E.size(); ++i) E[i]->finish(st[i], losses[i]);
    fwd_count = st[0].fwd_count;
    t = st[0].t;
    pre = st[0].next_pre;
  }
  return py::make_tuple(fwd_count, t, pre);
}

}  // namespace

void sl_register_engine(py::module& m) {
  m.def("tp_emulate_epoch", &tp_emulate_epoch, py::arg("executors"), py::arg("acts"), py::arg("labels"),
        py::arg("loss_rows"), py::arg("seed_base"), py::arg("fwd_count"), py::arg("t"), py::arg("pre"),
        py::arg("lookahead"));
  py::class_<ServerEpoch>(m, "ServerEpoch")
      .def(py::init<const py::dict&>())
      .def("run", &ServerEpoch::run, py::arg("acts"), py::arg("labels"), py::arg("loss_rows"), py::arg("seed_base"),
           py::arg("fwd_count"), py::arg("t"), py::arg("pre"), py::arg("lookahead"),
           py::arg("gscale") = py::none());
}
