// Python bindings for the gfx950 kernels (pybind11 module `splitlearning_amd._C`).
//
// Thin by design: validate shapes/dtypes/devices on the host (a kernel must never
// see an operand its grid does not assume), fetch the current HIP stream from the
// PyTorch-ROCm stream registry, and call the launcher.  All buffers are
// caller-allocated so the same calls can be captured into a HIP graph.
//
// Optimizer hyper-parameters travel as (kind, lr, beta1, beta2, eps, wd, momentum, t, dyn):
// kind 0 = write the gradient into s0, 1 = SGD(momentum), 2 = Adam (L2 weight decay);
// `dyn` != 0 is the device address of {step_size, inv_bc2_sqrt} used instead of t
// (graph replay).  Dropout seeds likewise: (seed, dseed) with dseed = device address
// of {seed_lo, seed_hi} or 0.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "common.h"
#include "fused.h"
#include "handoff.h"
#include "host.h"

namespace sl {
hipError_t conv_fwd(const void* x, bool x_u8, const int64_t* idx, int64_t row0, int B, const float* w,
                    const float* b, float* y, uint8_t* am, hipStream_t st, const int64_t* lab_in,
                    int64_t* lab_out, const ConvPending* pend);
hipError_t conv_local_step(const void* x, bool x_u8, const int64_t* idx, const int64_t* labels, int B, float* w,
                           float* b, float* slab, float* loss_rows, float* s0w, float* s1w, float* s0b, float* s1b,
                           SlOpt o, hipStream_t st);
hipError_t conv_local_epoch(const void* x, bool x_u8, const int64_t* order, int64_t n, int B, const int64_t* labels,
                            float* w, float* b, float* s0w, float* s1w, float* s0b, float* s1b, float* ws,
                            int64_t ws_elems, float* loss_rows, SlOpt (*opt)(void*, int64_t), void* optctx,
                            int64_t t0, hipStream_t st);
hipError_t conv_bwd_step(const float* dy, const float* y, const uint8_t* am, const void* x, bool x_u8,
                         const int64_t* idx, int B, float* w, float* b, float* slab, float* s0w, float* s1w,
                         float* s0b, float* s1b, SlOpt o, hipStream_t st, bool defer, const ConvPending* pend);
hipError_t conv_local_epoch_multi(const MultiAlice* al, int k, int B, SlOpt (*opt)(void*, int64_t), void* optctx,
                                  void* table, int64_t table_bytes, hipStream_t st);
size_t alice_step_desc_bytes();
hipError_t conv_apply(const ConvPending& p, float* w, float* b, hipStream_t st);
hipError_t conv_fwd_multi(const FrontFwdSet& set, int64_t chunk, hipStream_t st);
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
hipError_t gemm_nn_dgrad(const float* dZ, int ldz, const float* W, int ldw, const float* hprev, int ldh, float scale,
                         float* dX, int ldx, int M, int R, int K, float* ws, int64_t ws_elems, hipStream_t st);
hipError_t linear_fwd_partial(const float* X, int ldx, const float* W, int ldw, int M, int N, int K, float* ws,
                              int64_t ws_elems, int max_split, int* S_out, hipStream_t st);
hipError_t linear_wgrad_opt(const float* dZ, int ldz, const float* A, int lda, float* W, int ldw, float* s0,
                            float* s1, float* bias, float* sb0, float* sb1, int M, int N, int K, SlOpt o,
                            hipStream_t st);
hipError_t opt_flat(float* p, const float* g, float* s0, float* s1, int64_t n, SlOpt o, hipStream_t st);
hipError_t relu_mask(const float* d, const float* h, float scale, float* out, int64_t n, hipStream_t st);
hipError_t softmax_ce(const float* x, int ldx, const int64_t* y, int64_t ignore, float scale, float* loss_rows,
                      float* d, int ldd, int M, int C, hipStream_t st);
hipError_t eval_counters(const float* x, int ldx, const int64_t* y, int64_t omit, unsigned long long* counters,
                         int M, int C, hipStream_t st);
}  // namespace sl

namespace {

using OptT = c10::optional<at::Tensor>;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e)); }

void need_cuda(const at::Tensor& t, const char* name) { TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor"); }
void need_f32(const at::Tensor& t, const char* name) {
  need_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}
// row-major 2-D with unit column stride and 16-byte aligned rows (float4 loads)
void need_rows(const at::Tensor& t, const char* name) {
  need_f32(t, name);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be 2-D with unit column stride");
  TORCH_CHECK(t.stride(0) % 4 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0, name,
              " rows must be 16-byte aligned");
}
// 2-D with unit column stride (scalar access only)
void need_2d(const at::Tensor& t, const char* name) {
  need_f32(t, name);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be 2-D with unit column stride");
}
float* fptr(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

SlOpt make_opt(int64_t kind, double lr, double beta1, double beta2, double eps, double wd, double momentum,
               int64_t t, int64_t dyn) {
  if (kind == 2 && !dyn) TORCH_CHECK(t >= 1, "Adam step count must be >= 1");
  return sl::make_opt_raw((int)kind, lr, beta1, beta2, eps, wd, momentum, t, reinterpret_cast<const float*>(dyn));
}

Epi make_epi(const OptT& bias, bool relu, double drop_p, uint64_t seed, int64_t col_off, int64_t dseed) {
  return sl::make_epi_raw(fptr(bias), relu, drop_p, seed, (int)col_off, reinterpret_cast<const uint32_t*>(dseed));
}

#define OPT_ARGS int64_t kind, double lr, double beta1, double beta2, double eps, double wd, double momentum, \
                 int64_t t, int64_t dyn
#define OPT_PASS make_opt(kind, lr, beta1, beta2, eps, wd, momentum, t, dyn)

// ---------------------------------------------------------------- conv
void check_x(const at::Tensor& x) {
  need_cuda(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 784 == 0, "x must be contiguous [N,784]");
  TORCH_CHECK(x.scalar_type() == at::kByte || x.scalar_type() == at::kFloat, "x must be uint8 or float32");
}
void check_params(const at::Tensor& w, const at::Tensor& b) {
  need_f32(w, "w");
  need_f32(b, "b");
  TORCH_CHECK(w.numel() == 288 && b.numel() == 32 && w.is_contiguous() && b.is_contiguous(), "conv params 32x1x3x3");
}
void check_idx(const at::Tensor& idx, int64_t B) {
  need_cuda(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous() && idx.numel() >= B, "idx int64 [B]");
}
void check_slab(const at::Tensor& slab, int64_t B) {
  need_f32(slab, "slab");
  TORCH_CHECK(slab.is_contiguous() && slab.numel() >= B * 320, "slab workspace [B,320]");
}

// lab_in / lab_out (optional, together): the shard's labels [N] and the batch's gathered
// labels [B], written by the forward kernel (no separate index launch).
void conv_fwd(const at::Tensor& x, const at::Tensor& idx, int64_t B, const at::Tensor& w, const at::Tensor& b,
              at::Tensor& y, at::Tensor& am, const OptT& lab_in, const OptT& lab_out) {
  check_x(x);
  check_params(w, b);
  check_idx(idx, B);
  need_f32(y, "y");
  TORCH_CHECK(y.is_contiguous() && y.numel() >= B * 5408, "y too small");
  TORCH_CHECK(am.scalar_type() == at::kByte && am.is_contiguous() && am.numel() >= B * 5408, "am too small");
  TORCH_CHECK(lab_in.has_value() == lab_out.has_value(), "lab_in and lab_out go together");
  const int64_t* li = nullptr;
  int64_t* lo = nullptr;
  if (lab_in.has_value()) {
    need_cuda(*lab_in, "lab_in");
    need_cuda(*lab_out, "lab_out");
    TORCH_CHECK(lab_in->scalar_type() == at::kLong && lab_in->is_contiguous() && lab_in->numel() == x.numel() / 784,
                "lab_in int64 [N]");
    TORCH_CHECK(lab_out->scalar_type() == at::kLong && lab_out->is_contiguous() && lab_out->numel() >= B,
                "lab_out int64 [B]");
    li = lab_in->data_ptr<int64_t>();
    lo = lab_out->data_ptr<int64_t>();
  }
  check(sl::conv_fwd(x.data_ptr(), x.scalar_type() == at::kByte, idx.data_ptr<int64_t>(), 0, (int)B,
                     w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr<float>(), am.data_ptr<uint8_t>(),
                     cur_stream(), li, lo, nullptr),
        "conv_fwd");
}

ConvPending make_pending(const at::Tensor& slab, int64_t pB, at::Tensor& s0w, const OptT& s1w, at::Tensor& s0b,
                             const OptT& s1b, SlOpt o) {
  check_slab(slab, pB);
  TORCH_CHECK(pB >= 1, "pending batch");
  TORCH_CHECK(s0w.numel() == 288 && s0b.numel() == 32, "optimizer state");
  return ConvPending{slab.data_ptr<float>(), (int)pB, s0w.data_ptr<float>(), fptr(s1w), s0b.data_ptr<float>(),
                         fptr(s1b), o};
}

// Forward with a deferred optimizer step applied in-kernel (FrontEngine, split modes):
// (pslab, pB, states, opt of that step) is the last backward's update, not yet stored.
void conv_fwd_pending(const at::Tensor& x, const at::Tensor& idx, int64_t B, const at::Tensor& w, const at::Tensor& b,
                      at::Tensor& y, at::Tensor& am, const at::Tensor& lab_in, at::Tensor& lab_out,
                      const at::Tensor& pslab, int64_t pB, at::Tensor& s0w, const OptT& s1w, at::Tensor& s0b,
                      const OptT& s1b, OPT_ARGS) {
  check_x(x);
  check_params(w, b);
  check_idx(idx, B);
  need_f32(y, "y");
  TORCH_CHECK(y.is_contiguous() && y.numel() >= B * 5408, "y too small");
  TORCH_CHECK(am.scalar_type() == at::kByte && am.is_contiguous() && am.numel() >= B * 5408, "am too small");
  need_cuda(lab_in, "lab_in");
  need_cuda(lab_out, "lab_out");
  TORCH_CHECK(lab_in.scalar_type() == at::kLong && lab_in.is_contiguous() && lab_in.numel() == x.numel() / 784,
              "lab_in int64 [N]");
  TORCH_CHECK(lab_out.scalar_type() == at::kLong && lab_out.is_contiguous() && lab_out.numel() >= B,
              "lab_out int64 [B]");
  const ConvPending p = make_pending(pslab, pB, s0w, s1w, s0b, s1b, OPT_PASS);
  check(sl::conv_fwd(x.data_ptr(), x.scalar_type() == at::kByte, idx.data_ptr<int64_t>(), 0, (int)B,
                     w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr<float>(), am.data_ptr<uint8_t>(),
                     cur_stream(), lab_in.data_ptr<int64_t>(), lab_out.data_ptr<int64_t>(), &p),
        "conv_fwd_pending");
}

// SISA local step: fused gather+conv+pool+softmax-CE(5408)+dW partials, then reduce+optimizer.
void conv_local_step(const at::Tensor& x, const at::Tensor& idx, const at::Tensor& labels, int64_t B, at::Tensor& w,
                     at::Tensor& b, at::Tensor& slab, at::Tensor& loss_rows, at::Tensor& s0w, const OptT& s1w,
                     at::Tensor& s0b, const OptT& s1b, OPT_ARGS) {
  check_x(x);
  check_params(w, b);
  check_idx(idx, B);
  check_slab(slab, B);
  need_cuda(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == x.numel() / 784, "labels int64 [N]");
  need_f32(loss_rows, "loss_rows");
  TORCH_CHECK(loss_rows.numel() >= B, "loss_rows");
  TORCH_CHECK(s0w.numel() == 288 && s0b.numel() == 32, "optimizer state");
  check(sl::conv_local_step(x.data_ptr(), x.scalar_type() == at::kByte, idx.data_ptr<int64_t>(),
                            labels.data_ptr<int64_t>(), (int)B, w.data_ptr<float>(), b.data_ptr<float>(),
                            slab.data_ptr<float>(), loss_rows.data_ptr<float>(), s0w.data_ptr<float>(), fptr(s1w),
                            s0b.data_ptr<float>(), fptr(s1b), OPT_PASS, cur_stream()),
        "conv_local_step");
}

struct EpochOpt {
  int64_t kind;
  double lr, beta1, beta2, eps, wd, momentum;
};
SlOpt epoch_opt(void* ctx, int64_t t) {
  const EpochOpt& e = *static_cast<const EpochOpt*>(ctx);
  return make_opt(e.kind, e.lr, e.beta1, e.beta2, e.eps, e.wd, e.momentum, t, 0);
}

// A whole SISA local epoch: ceil(n/B) client steps over `order` (the last one partial, like
// DataLoader(drop_last=False)), optimizer steps t0, t0+1, ...  One launch per step: each
// step's kernel applies the previous step's optimizer update in its prologue
// (conv.hip: conv_local_epoch).
void conv_local_epoch(const at::Tensor& x, const at::Tensor& order, const at::Tensor& labels, int64_t B,
                      at::Tensor& w, at::Tensor& b, at::Tensor& slab, at::Tensor& loss_rows, at::Tensor& s0w,
                      const OptT& s1w, at::Tensor& s0b, const OptT& s1b, int64_t kind, double lr, double beta1,
                      double beta2, double eps, double wd, double momentum, int64_t t0, at::Tensor& ws) {
  check_x(x);
  check_params(w, b);
  need_cuda(order, "order");
  TORCH_CHECK(order.scalar_type() == at::kLong && order.is_contiguous() && order.dim() == 1, "order int64 [n]");
  const int64_t n = order.numel();
  TORCH_CHECK(B >= 1 && B <= 4096, "batch size");
  check_slab(slab, B);
  need_cuda(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == x.numel() / 784, "labels int64 [N]");
  need_f32(loss_rows, "loss_rows");
  TORCH_CHECK(loss_rows.is_contiguous() && loss_rows.numel() >= n, "loss_rows [n]");
  TORCH_CHECK(s0w.numel() == 288 && s0b.numel() == 32, "optimizer state");
  need_f32(ws, "ws");
  TORCH_CHECK(ws.is_contiguous(), "ws contiguous");
  TORCH_CHECK(kind == 1 || kind == 2, "local epoch: SGD-momentum or Adam");
  const hipStream_t st = cur_stream();
  EpochOpt ctx{kind, lr, beta1, beta2, eps, wd, momentum};
  check(sl::conv_local_epoch(x.data_ptr(), x.scalar_type() == at::kByte, order.data_ptr<int64_t>(), n, (int)B,
                             labels.data_ptr<int64_t>(), w.data_ptr<float>(), b.data_ptr<float>(),
                             s0w.data_ptr<float>(), fptr(s1w), s0b.data_ptr<float>(), fptr(s1b), ws.data_ptr<float>(),
                             ws.numel(), loss_rows.data_ptr<float>(), &epoch_opt, &ctx, t0, st),
        "conv_local_epoch");
}

// Local epochs of k co-located Alices stepped together, one launch per step for all of
// them (conv.hip: conv_local_epoch_multi).  alices: [(x, order, labels, w, b, s0w, s1w, s0b,
// s1b, ws, loss_rows, t0)]; every Alice shares the optimizer hyper-parameters.  `table`:
// uint8 GPU workspace >= table_bytes(k, max steps).
void conv_local_epoch_multi(py::list alices, int64_t B, int64_t kind, double lr, double beta1, double beta2, double eps,
                            double wd, double momentum, at::Tensor& table) {
  const int k = (int)alices.size();
  TORCH_CHECK(k >= 1 && k <= 64, "1..64 co-located Alices");
  TORCH_CHECK(B >= 1 && B <= 1024, "batch size");
  TORCH_CHECK(kind == 1 || kind == 2, "local epoch: SGD-momentum or Adam");
  need_cuda(table, "table");
  TORCH_CHECK(table.scalar_type() == at::kByte && table.is_contiguous(), "table uint8 workspace");
  std::vector<MultiAlice> al(k);
  for (int a = 0; a < k; ++a) {
    auto t = alices[a].cast<py::tuple>();
    TORCH_CHECK(t.size() == 12, "alice tuple (x, order, labels, w, b, s0w, s1w, s0b, s1b, ws, loss_rows, t0)");
    auto x = t[0].cast<at::Tensor>();
    auto order = t[1].cast<at::Tensor>();
    auto labels = t[2].cast<at::Tensor>();
    auto w = t[3].cast<at::Tensor>();
    auto b = t[4].cast<at::Tensor>();
    auto s0w = t[5].cast<at::Tensor>();
    auto s1w = t[6].cast<OptT>();
    auto s0b = t[7].cast<at::Tensor>();
    auto s1b = t[8].cast<OptT>();
    auto ws = t[9].cast<at::Tensor>();
    auto loss = t[10].cast<at::Tensor>();
    check_x(x);
    TORCH_CHECK(x.scalar_type() == at::kByte, "co-located epochs read uint8 shards");
    check_params(w, b);
    need_cuda(order, "order");
    TORCH_CHECK(order.scalar_type() == at::kLong && order.is_contiguous() && order.dim() == 1, "order int64 [n]");
    need_cuda(labels, "labels");
    TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == x.numel() / 784,
                "labels int64 [N]");
    TORCH_CHECK(s0w.numel() == 288 && s0b.numel() == 32, "optimizer state");
    need_f32(ws, "ws");
    TORCH_CHECK(ws.is_contiguous() && ws.numel() >= 2 * B * 320 + 2 * 960, "ws");
    need_f32(loss, "loss_rows");
    TORCH_CHECK(loss.is_contiguous() && loss.numel() >= order.numel(), "loss_rows [n]");
    al[a] = MultiAlice{x.data_ptr<uint8_t>(), order.data_ptr<int64_t>(), order.numel(), labels.data_ptr<int64_t>(),
                           w.data_ptr<float>(), b.data_ptr<float>(), s0w.data_ptr<float>(), fptr(s1w),
                           s0b.data_ptr<float>(), fptr(s1b), ws.data_ptr<float>(), ws.numel(),
                           loss.data_ptr<float>(), t[11].cast<int64_t>()};
    if (kind == 2) TORCH_CHECK(al[a].s1w && al[a].s1b, "Adam second moments");
  }
  EpochOpt ctx{kind, lr, beta1, beta2, eps, wd, momentum};
  check(sl::conv_local_epoch_multi(al.data(), k, (int)B, &epoch_opt, &ctx, table.data_ptr(), table.numel(),
                                   cur_stream()),
        "conv_local_epoch_multi");
}

// Frozen-front forwards of up to 16 co-located Alices, one launch per `chunk` rows for all of
// them (conv.hip: conv_fwd_multi).  alices: [(x uint8 [N, 784], idx int64 [n] or None (rows
// 0 .. n), n, w, b, y [n, 5408])].
void conv_fwd_multi(py::list alices, int64_t chunk) {
  const int k = (int)alices.size();
  TORCH_CHECK(k >= 1 && k <= kFrontFwdMax, "1..16 Alices per launch");
  TORCH_CHECK(chunk >= 1 && chunk <= 65535, "chunk rows");
  FrontFwdSet set{};
  set.k = k;
  for (int a = 0; a < k; ++a) {
    auto t = alices[a].cast<py::tuple>();
    TORCH_CHECK(t.size() == 6, "alice tuple (x, idx, n, w, b, y)");
    auto x = t[0].cast<at::Tensor>();
    auto idx = t[1].cast<OptT>();
    const int64_t n = t[2].cast<int64_t>();
    auto w = t[3].cast<at::Tensor>();
    auto b = t[4].cast<at::Tensor>();
    auto y = t[5].cast<at::Tensor>();
    check_x(x);
    TORCH_CHECK(x.scalar_type() == at::kByte, "uint8 shards");
    check_params(w, b);
    TORCH_CHECK(n >= 0, "n");
    if (idx.has_value()) {
      check_idx(*idx, n);
    } else {
      TORCH_CHECK(n <= x.numel() / 784, "rows beyond the shard");
    }
    need_f32(y, "y");
    TORCH_CHECK(y.is_contiguous() && y.numel() >= n * 5408, "y [n, 5408]");
    set.d[a] = FrontFwdDesc{x.data_ptr<uint8_t>(), idx.has_value() ? idx->data_ptr<int64_t>() : nullptr, n,
                            w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr<float>()};
  }
  check(sl::conv_fwd_multi(set, chunk, cur_stream()), "conv_fwd_multi");
}

// Split-mode client backward: dW partials from the cut gradient, then reduce+optimizer.
void conv_bwd_step(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& am, const at::Tensor& x,
                   const at::Tensor& idx, int64_t B, at::Tensor& w, at::Tensor& b, at::Tensor& slab, at::Tensor& s0w,
                   const OptT& s1w, at::Tensor& s0b, const OptT& s1b, OPT_ARGS) {
  check_x(x);
  check_params(w, b);
  check_idx(idx, B);
  check_slab(slab, B);
  need_f32(dy, "dy");
  need_f32(y, "y");
  TORCH_CHECK(dy.is_contiguous() && y.is_contiguous() && dy.numel() >= B * 5408 && y.numel() >= B * 5408, "dy/y");
  TORCH_CHECK(am.scalar_type() == at::kByte && am.is_contiguous() && am.numel() >= B * 5408, "am");
  TORCH_CHECK(s0w.numel() == 288 && s0b.numel() == 32, "optimizer state");
  check(sl::conv_bwd_step(dy.data_ptr<float>(), y.data_ptr<float>(), am.data_ptr<uint8_t>(), x.data_ptr(),
                          x.scalar_type() == at::kByte, idx.data_ptr<int64_t>(), (int)B, w.data_ptr<float>(),
                          b.data_ptr<float>(), slab.data_ptr<float>(), s0w.data_ptr<float>(), fptr(s1w),
                          s0b.data_ptr<float>(), fptr(s1b), OPT_PASS, cur_stream(), false, nullptr),
        "conv_bwd_step");
}

// Deferred-update backward: this step's dW/db partials into `slab` (no update launch);
// workgroup 0 stores the pending update of the previous step (pslab / pB / its opt), if any.
void conv_bwd_defer(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& am, const at::Tensor& x,
                    const at::Tensor& idx, int64_t B, at::Tensor& w, at::Tensor& b, at::Tensor& slab, const OptT& pslab,
                    int64_t pB, at::Tensor& s0w, const OptT& s1w, at::Tensor& s0b, const OptT& s1b, OPT_ARGS) {
  check_x(x);
  check_params(w, b);
  check_idx(idx, B);
  check_slab(slab, B);
  need_f32(dy, "dy");
  need_f32(y, "y");
  TORCH_CHECK(dy.is_contiguous() && y.is_contiguous() && dy.numel() >= B * 5408 && y.numel() >= B * 5408, "dy/y");
  TORCH_CHECK(am.scalar_type() == at::kByte && am.is_contiguous() && am.numel() >= B * 5408, "am");
  TORCH_CHECK(s0w.numel() == 288 && s0b.numel() == 32, "optimizer state");
  const bool has = pslab.has_value() && pslab->defined();
  ConvPending p{};
  if (has) {
    TORCH_CHECK(pslab->data_ptr<float>() != slab.data_ptr<float>(), "pending and new slabs must differ");
    p = make_pending(*pslab, pB, s0w, s1w, s0b, s1b, OPT_PASS);
  }
  check(sl::conv_bwd_step(dy.data_ptr<float>(), y.data_ptr<float>(), am.data_ptr<uint8_t>(), x.data_ptr(),
                          x.scalar_type() == at::kByte, idx.data_ptr<int64_t>(), (int)B, w.data_ptr<float>(),
                          b.data_ptr<float>(), slab.data_ptr<float>(), s0w.data_ptr<float>(), fptr(s1w),
                          s0b.data_ptr<float>(), fptr(s1b), SlOpt{}, cur_stream(), true, has ? &p : nullptr),
        "conv_bwd_defer");
}

// U-shape head (Linear + CE) forward, data gradient and optimizer step in one launch.
void head_step(const at::Tensor& X, at::Tensor& W, const OptT& b, const at::Tensor& y, int64_t ignore, double scale,
               bool mask_dx, at::Tensor& loss_rows, at::Tensor& dX, at::Tensor& s0w, const OptT& s1w, const OptT& s0b,
               const OptT& s1b, OPT_ARGS) {
  need_rows(X, "X");
  need_rows(W, "W");
  const int64_t M = X.size(0), K = X.size(1), C = W.size(0);
  TORCH_CHECK(X.is_contiguous() && W.is_contiguous() && W.size(1) == K, "X [M,K], W [C,K] contiguous");
  TORCH_CHECK(M * K <= 4096 && C * K <= 4096 && M * C <= 1024, "head_step: layer too large for one workgroup");
  need_cuda(y, "y");
  TORCH_CHECK(y.scalar_type() == at::kLong && y.numel() == M, "labels int64 [M]");
  need_f32(loss_rows, "loss_rows");
  need_f32(dX, "dX");
  TORCH_CHECK(loss_rows.numel() >= M && dX.is_contiguous() && dX.numel() == M * K, "outputs");
  TORCH_CHECK(s0w.numel() == C * K && s0w.is_contiguous(), "state");
  if (b.has_value() && b->defined()) TORCH_CHECK(b->numel() == C && s0b.has_value(), "bias state");
  check(sl::head_step(X.data_ptr<float>(), W.data_ptr<float>(), fptr(b), y.data_ptr<int64_t>(), ignore, (float)scale,
                      loss_rows.data_ptr<float>(), dX.data_ptr<float>(), s0w.data_ptr<float>(), fptr(s1w), fptr(s0b),
                      fptr(s1b), (int)M, (int)K, (int)C, OPT_PASS, mask_dx, cur_stream()),
        "head_step");
}

// Store a deferred update (FrontEngine.flush).
void conv_apply(const at::Tensor& pslab, int64_t pB, at::Tensor& w, at::Tensor& b, at::Tensor& s0w, const OptT& s1w,
                at::Tensor& s0b, const OptT& s1b, OPT_ARGS) {
  check_params(w, b);
  const ConvPending p = make_pending(pslab, pB, s0w, s1w, s0b, s1b, OPT_PASS);
  check(sl::conv_apply(p, w.data_ptr<float>(), b.data_ptr<float>(), cur_stream()), "conv_apply");
}

// ---------------------------------------------------------------- linear
void linear_fwd(const at::Tensor& X, const at::Tensor& W, const OptT& bias, at::Tensor& Y, bool relu, double drop_p,
                uint64_t seed, int64_t col_off, int64_t dseed, const OptT& ws) {
  need_rows(X, "X");
  need_rows(W, "W");
  need_2d(Y, "Y");
  const int64_t M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K && K % 4 == 0, "W must be [N,K] with K % 4 == 0");
  TORCH_CHECK(Y.size(0) == M && Y.size(1) == N, "Y must be [M,N]");
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "bias [N]");
  float* wp = nullptr;
  int64_t wn = 0;
  if (ws.has_value() && ws->defined()) {
    need_f32(*ws, "ws");
    TORCH_CHECK(ws->is_contiguous(), "ws contiguous");
    wp = ws->data_ptr<float>();
    wn = ws->numel();
  }
  check(sl::linear_fwd(X.data_ptr<float>(), (int)X.stride(0), W.data_ptr<float>(), (int)W.stride(0),
                       Y.data_ptr<float>(), (int)Y.stride(0), (int)M, (int)N, (int)K,
                       make_epi(bias, relu, drop_p, seed, col_off, dseed), wp, wn, cur_stream()),
        "linear_fwd");
}

// P: [M, N] pre-activations, or [S, M, N] contiguous split-K partial slabs (summed here).
void linear_epilogue(const at::Tensor& P, const OptT& bias, at::Tensor& Y, bool relu, double drop_p, uint64_t seed,
                     int64_t col_off, int64_t dseed) {
  need_2d(Y, "Y");
  int S = 1;
  int64_t slab = 0;
  if (P.dim() == 3) {
    need_f32(P, "P");
    TORCH_CHECK(P.is_contiguous() && P.size(1) == Y.size(0) && P.size(2) == Y.size(1), "P [S,M,N]");
    S = (int)P.size(0);
    slab = P.size(1) * P.size(2);
  } else {
    need_2d(P, "P");
    TORCH_CHECK(P.sizes() == Y.sizes(), "P/Y shape");
  }
  const int64_t M = Y.size(0), N = Y.size(1);
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == N, "bias [N]");
  check(sl::linear_epilogue(P.data_ptr<float>(), (int)P.stride(P.dim() - 2), Y.data_ptr<float>(), (int)Y.stride(0),
                            (int)M, (int)N, make_epi(bias, relu, drop_p, seed, col_off, dseed), S, slab, cur_stream()),
        "linear_epilogue");
}

void linear_dgrad(const at::Tensor& dZ, const at::Tensor& W, const OptT& hprev, double scale, at::Tensor& dX,
                  const OptT& ws) {
  need_2d(dZ, "dZ");
  need_rows(W, "W");
  need_2d(dX, "dX");
  const int64_t M = dZ.size(0), N = dZ.size(1), K = W.size(1);
  TORCH_CHECK(W.size(0) == N && K % 4 == 0, "W must be [N,K]");
  TORCH_CHECK(dX.size(0) == M && dX.size(1) == K, "dX must be [M,K]");
  const float* hp = nullptr;
  int ldh = 0;
  if (hprev.has_value() && hprev->defined()) {
    need_2d(*hprev, "hprev");
    TORCH_CHECK(hprev->size(0) == M && hprev->size(1) == K, "hprev shape");
    hp = hprev->data_ptr<float>();
    ldh = (int)hprev->stride(0);
  }
  float* wp = nullptr;
  int64_t wn = 0;
  if (ws.has_value() && ws->defined()) {
    need_f32(*ws, "ws");
    TORCH_CHECK(ws->is_contiguous(), "ws contiguous");
    wp = ws->data_ptr<float>();
    wn = ws->numel();
  }
  check(sl::linear_dgrad(dZ.data_ptr<float>(), (int)dZ.stride(0), W.data_ptr<float>(), (int)W.stride(0), hp, ldh,
                         (float)scale, dX.data_ptr<float>(), (int)dX.stride(0), wp, wn, (int)M, (int)N, (int)K,
                         cur_stream()),
        "linear_dgrad");
}

// the data gradient of many rows on the in-tree NN-layout MFMA GEMM (csrc/gemm.hip)
void gemm_nn_dgrad(const at::Tensor& dZ, const at::Tensor& W, const OptT& hprev, double scale, at::Tensor& dX,
                   const OptT& ws) {
  need_2d(dZ, "dZ");
  need_rows(W, "W");
  need_2d(dX, "dX");
  const int64_t M = dZ.size(0), N = dZ.size(1), K = W.size(1);
  TORCH_CHECK(W.size(0) == N && K % 4 == 0 && N % 4 == 0, "W must be [N,K], N and K % 4 == 0");
  TORCH_CHECK(dX.size(0) == M && dX.size(1) == K, "dX must be [M,K]");
  TORCH_CHECK(dZ.stride(0) % 4 == 0 && W.stride(0) % 4 == 0, "rows 16-B aligned");
  const float* hp = nullptr;
  int ldh = 0;
  if (hprev.has_value() && hprev->defined()) {
    need_2d(*hprev, "hprev");
    TORCH_CHECK(hprev->size(0) == M && hprev->size(1) == K, "hprev shape");
    hp = hprev->data_ptr<float>();
    ldh = (int)hprev->stride(0);
  }
  float* wp = nullptr;
  int64_t wn = 0;
  if (ws.has_value() && ws->defined()) {
    need_f32(*ws, "ws");
    TORCH_CHECK(ws->is_contiguous(), "ws contiguous");
    wp = ws->data_ptr<float>();
    wn = ws->numel();
  }
  check(sl::gemm_nn_dgrad(dZ.data_ptr<float>(), (int)dZ.stride(0), W.data_ptr<float>(), (int)W.stride(0), hp, ldh,
                          (float)scale, dX.data_ptr<float>(), (int)dX.stride(0), (int)M, (int)N, (int)K, wp, wn,
                          cur_stream()),
        "gemm_nn_dgrad");
}

void linear_wgrad_opt(const at::Tensor& dZ, const at::Tensor& A, at::Tensor& W, at::Tensor& s0, const OptT& s1,
                      const OptT& bias, const OptT& sb0, const OptT& sb1, OPT_ARGS) {
  need_2d(dZ, "dZ");
  need_rows(A, "A");
  need_rows(W, "W");
  need_rows(s0, "s0");
  const int64_t M = dZ.size(0), N = dZ.size(1), K = A.size(1);
  TORCH_CHECK(A.size(0) == M && W.size(0) == N && W.size(1) == K && K % 4 == 0, "shapes");
  TORCH_CHECK(s0.sizes() == W.sizes() && s0.stride(0) == W.stride(0), "s0 like W");
  if (s1.has_value() && s1->defined()) TORCH_CHECK(s1->sizes() == W.sizes() && s1->stride(0) == W.stride(0), "s1");
  if (kind == 2) TORCH_CHECK(s1.has_value() && s1->defined(), "Adam needs s1");
  if (bias.has_value() && bias->defined())
    TORCH_CHECK(bias->numel() == N && sb0.has_value() && sb0->numel() == N, "bias state");
  check(sl::linear_wgrad_opt(dZ.data_ptr<float>(), (int)dZ.stride(0), A.data_ptr<float>(), (int)A.stride(0),
                             W.data_ptr<float>(), (int)W.stride(0), s0.data_ptr<float>(), fptr(s1), fptr(bias),
                             fptr(sb0), fptr(sb1), (int)M, (int)N, (int)K, OPT_PASS, cur_stream()),
        "linear_wgrad_opt");
}

void opt_flat(at::Tensor& p, const at::Tensor& g, at::Tensor& s0, const OptT& s1, OPT_ARGS) {
  need_f32(p, "p");
  need_f32(g, "g");
  need_f32(s0, "s0");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && s0.is_contiguous(), "contiguous");
  TORCH_CHECK(g.numel() == p.numel() && s0.numel() == p.numel(), "sizes");
  check(sl::opt_flat(p.data_ptr<float>(), g.data_ptr<float>(), s0.data_ptr<float>(), fptr(s1), p.numel(), OPT_PASS,
                     cur_stream()),
        "opt_flat");
}

// ---------------------------------------------------------------- loss / metrics
void softmax_ce(const at::Tensor& x, const at::Tensor& y, int64_t ignore, double scale, at::Tensor& loss_rows,
                const OptT& d) {
  need_2d(x, "logits");
  const int64_t M = x.size(0), C = x.size(1);
  need_cuda(y, "labels");
  TORCH_CHECK(y.scalar_type() == at::kLong && y.numel() == M && y.is_contiguous(), "labels int64 [M]");
  need_f32(loss_rows, "loss_rows");
  TORCH_CHECK(loss_rows.numel() >= M, "loss_rows");
  float* dp = nullptr;
  int ldd = 0;
  if (d.has_value() && d->defined()) {
    need_2d(*d, "dlogits");
    TORCH_CHECK(d->size(0) == M && d->size(1) == C, "dlogits shape");
    dp = d->data_ptr<float>();
    ldd = (int)d->stride(0);
  }
  check(sl::softmax_ce(x.data_ptr<float>(), (int)x.stride(0), y.data_ptr<int64_t>(), ignore, (float)scale,
                       loss_rows.data_ptr<float>(), dp, ldd, (int)M, (int)C, cur_stream()),
        "softmax_ce");
}

void relu_mask(const at::Tensor& d, const at::Tensor& h, double scale, at::Tensor& out) {
  need_f32(d, "d");
  need_f32(h, "h");
  need_f32(out, "out");
  TORCH_CHECK(d.is_contiguous() && h.is_contiguous() && out.is_contiguous() && d.numel() == h.numel() &&
                  out.numel() == d.numel(),
              "relu_mask: contiguous tensors of one size");
  check(sl::relu_mask(d.data_ptr<float>(), h.data_ptr<float>(), (float)scale, out.data_ptr<float>(), d.numel(),
                      cur_stream()),
        "relu_mask");
}

void eval_counters(const at::Tensor& x, const at::Tensor& y, int64_t omit, at::Tensor& counters) {
  need_2d(x, "logits");
  TORCH_CHECK(y.scalar_type() == at::kLong && y.numel() == x.size(0) && y.is_contiguous(), "labels");
  TORCH_CHECK(counters.scalar_type() == at::kLong && counters.numel() >= 6 && counters.is_contiguous(), "counters");
  need_cuda(counters, "counters");
  check(sl::eval_counters(x.data_ptr<float>(), (int)x.stride(0), y.data_ptr<int64_t>(), omit,
                          reinterpret_cast<unsigned long long*>(counters.data_ptr<int64_t>()), (int)x.size(0),
                          (int)x.size(1), cur_stream()),
        "eval_counters");
}

// Partial products into a workspace; return the number of slabs S (result = ws[:S*M*cols]).
int64_t linear_fwd_partial(const at::Tensor& X, const at::Tensor& W, at::Tensor& ws, int64_t max_split) {
  need_rows(X, "X");
  need_rows(W, "W");
  need_f32(ws, "ws");
  TORCH_CHECK(ws.is_contiguous(), "ws contiguous");
  const int64_t M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K && K % 4 == 0, "W must be [N,K] with K % 4 == 0");
  int S = 1;
  check(sl::linear_fwd_partial(X.data_ptr<float>(), (int)X.stride(0), W.data_ptr<float>(), (int)W.stride(0), (int)M,
                               (int)N, (int)K, ws.data_ptr<float>(), ws.numel(), (int)max_split, &S, cur_stream()),
        "linear_fwd_partial");
  return S;
}

// ---------------------------------------------------------------- fused server step
// P2: fc2 partial sums, [S2, M, N2] split-K slabs or a reduced [M, N2] tensor.
void server_head3(const at::Tensor& P2, const OptT& b2, bool relu2, double drop2, uint64_t seed2, int64_t dseed2,
                  const at::Tensor& W3, const OptT& b3, const at::Tensor& y, int64_t ignore, double scale,
                  at::Tensor& h2, at::Tensor& dlog, at::Tensor& dz2, at::Tensor& loss_rows, at::Tensor& ws, int64_t G,
                  const OptT& gscale) {
  need_f32(P2, "P2");
  TORCH_CHECK(P2.is_contiguous() && (P2.dim() == 2 || P2.dim() == 3), "P2 [S,M,N2] or [M,N2] contiguous");
  const int64_t S2 = P2.dim() == 3 ? P2.size(0) : 1;
  const int64_t M = P2.size(P2.dim() - 2), N2 = P2.size(P2.dim() - 1);
  need_rows(W3, "W3");
  const int64_t C = W3.size(0);
  TORCH_CHECK(W3.size(1) == N2 && N2 % 4 == 0 && W3.stride(0) % 4 == 0 && C <= 4096, "W3 [C, N2], N2 % 4 == 0");
  need_f32(ws, "ws");
  TORCH_CHECK(ws.is_contiguous() && ws.numel() >= (int64_t)sl::head3_slices((int)N2) * M * C, "head workspace");
  need_cuda(y, "labels");
  TORCH_CHECK(G >= 1 && C % G == 0, "C % groups");
  TORCH_CHECK(y.scalar_type() == at::kLong && y.numel() == M * G && y.is_contiguous(), "labels int64 [M, groups]");
  if (gscale.has_value() && gscale->defined()) {
    need_f32(*gscale, "gscale");
    TORCH_CHECK(gscale->is_contiguous() && gscale->numel() == M * G, "gscale [M, groups]");
  }
  for (auto* t : {&h2, &dz2}) {
    need_f32(*t, "h2/dz2");
    TORCH_CHECK(t->is_contiguous() && t->size(0) == M && t->size(1) == N2, "h2/dz2 [M,N2]");
  }
  need_f32(dlog, "dlog");
  TORCH_CHECK(dlog.is_contiguous() && dlog.size(0) == M && dlog.size(1) == C, "dlog [M,C]");
  need_f32(loss_rows, "loss_rows");
  TORCH_CHECK(loss_rows.numel() >= M * G, "loss_rows [M, groups]");
  check(sl::server_head3(P2.data_ptr<float>(), (int)S2, M * N2, make_epi(b2, relu2, drop2, seed2, 0, dseed2),
                         W3.data_ptr<float>(), (int)W3.stride(0), fptr(b3), y.data_ptr<int64_t>(), ignore,
                         (float)scale, h2.data_ptr<float>(), dlog.data_ptr<float>(), dz2.data_ptr<float>(),
                         loss_rows.data_ptr<float>(), ws.data_ptr<float>(), ws.numel(), (int)M, (int)N2, (int)C,
                         cur_stream(), nullptr, (int)G, fptr(gscale)),
        "server_head3");
}

// layers: up to 3 tuples (dz, A, W, s0, s1, bias, sb0, sb1).
// xn / pn (optional): next batch [mn, K0] -> its split-K partial pre-activations of layer 0
// with the updated weights, pn = [ceil(K0/256), mn, N0].
void wgrad_group(const std::vector<py::tuple>& layers, int64_t M, const OptT& xn, const OptT& pn, OPT_ARGS) {
  TORCH_CHECK(!layers.empty() && layers.size() <= 3, "1..3 layers");
  sl::WgGroup g{};
  g.n = (int)layers.size();
  for (size_t i = 0; i < layers.size(); ++i) {
    const py::tuple& L = layers[i];
    TORCH_CHECK(L.size() == 8, "layer tuple (dz, A, W, s0, s1, bias, sb0, sb1)");
    auto opt = [&](int j) -> OptT { return L[j].is_none() ? OptT() : OptT(L[j].cast<at::Tensor>()); };
    const at::Tensor dz = L[0].cast<at::Tensor>();
    const at::Tensor A = L[1].cast<at::Tensor>();
    at::Tensor W = L[2].cast<at::Tensor>();
    at::Tensor s0 = L[3].cast<at::Tensor>();
    need_rows(A, "A");
    need_rows(W, "W");
    need_rows(s0, "s0");
    const int64_t N = W.size(0), K = W.size(1);
    TORCH_CHECK(A.size(0) == M && A.size(1) == K && K % 4 == 0, "A [M,K]");
    TORCH_CHECK(s0.sizes() == W.sizes() && s0.stride(0) == W.stride(0), "s0 like W");
    OptT s1 = opt(4), bias = opt(5), sb0 = opt(6), sb1 = opt(7);
    if (kind == 2) TORCH_CHECK(s1.has_value() && s1->sizes() == W.sizes() && s1->stride(0) == W.stride(0), "s1");
    if (bias.has_value()) TORCH_CHECK(bias->numel() == N && sb0.has_value() && sb0->numel() == N, "bias state");
    sl::WgDesc& d = g.d[i];
    need_2d(dz, "dz");
    TORCH_CHECK(dz.size(0) == M && dz.size(1) == N, "dz [M,N]");
    d.dz = dz.data_ptr<float>();
    d.ldz = (int)dz.stride(0);
    d.A = A.data_ptr<float>();
    d.lda = (int)A.stride(0);
    d.W = W.data_ptr<float>();
    d.ldw = (int)W.stride(0);
    d.s0 = s0.data_ptr<float>();
    d.s1 = fptr(s1);
    d.bias = fptr(bias);
    d.sb0 = fptr(sb0);
    d.sb1 = fptr(sb1);
    d.N = (int)N;
    d.K = (int)K;
  }
  if (xn.has_value() && xn->defined()) {
    TORCH_CHECK(pn.has_value() && pn->defined(), "pn needed with xn");
    need_rows(*xn, "xn");
    need_f32(*pn, "pn");
    const int64_t K0 = g.d[0].K, N0 = g.d[0].N, mn = xn->size(0);
    TORCH_CHECK(xn->size(1) == K0 && mn >= 1 && mn <= 64, "xn [mn<=64, K0]");
    TORCH_CHECK(pn->is_contiguous() && pn->numel() >= (K0 + 255) / 256 * mn * N0, "pn [K0/256, mn, N0]");
    g.xn = xn->data_ptr<float>();
    g.ldxn = (int)xn->stride(0);
    g.mn = (int)mn;
    g.pn = pn->data_ptr<float>();
  }
  check(sl::wgrad_group(g, (int)M, OPT_PASS, cur_stream()), "wgrad_group");
}

}  // namespace

void sl_register_comm(pybind11::module& m);
void sl_register_engine(pybind11::module& m);
void sl_register_split(pybind11::module& m);
void sl_register_resident(pybind11::module& m);
void sl_register_hybrid(pybind11::module& m);
void sl_register_vanilla(pybind11::module& m);
void sl_register_ushape(pybind11::module& m);

PYBIND11_MODULE(_C, m) {
  m.doc() = "splitlearning_amd gfx950 (MI355X) HIP kernels";
  sl_register_comm(m);
  sl_register_engine(m);
  sl_register_split(m);
  sl_register_resident(m);
  sl_register_hybrid(m);
  sl_register_vanilla(m);
  sl_register_ushape(m);
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_local_step", &conv_local_step);
  m.def("conv_bwd_step", &conv_bwd_step);
  m.def("conv_bwd_defer", &conv_bwd_defer);
  m.def("conv_fwd_pending", &conv_fwd_pending);
  m.def("conv_apply", &conv_apply);
  m.def("head_step", &head_step);
  m.def("conv_local_epoch", &conv_local_epoch);
  m.def("conv_local_epoch_multi", &conv_local_epoch_multi);
  m.def("conv_fwd_multi", &conv_fwd_multi);
  m.def("alice_step_desc_bytes", []() { return (int64_t)sl::alice_step_desc_bytes(); });
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_epilogue", &linear_epilogue);
  m.def("linear_dgrad", &linear_dgrad);
  m.def("gemm_nn_dgrad", &gemm_nn_dgrad);
  m.def("linear_wgrad_opt", &linear_wgrad_opt);
  m.def("opt_flat", &opt_flat);
  m.def("softmax_ce", &softmax_ce);
  m.def("eval_counters", &eval_counters);
  m.def("relu_mask", &relu_mask);
  m.def("server_head3", &server_head3);
  m.def("head3_slices", [](int64_t n2) { return (int64_t)sl::head3_slices((int)n2); });
  m.def("linear_fwd_partial", &linear_fwd_partial);
  m.def("wgrad_group", &wgrad_group);
  // Kernel-variant slots for A/B runs of work in progress (0 = the default everywhere).  A
  // slot lives only while its alternative is being measured; the losers are removed with the
  // numbers kept in docs/PERF.md.  In use:
  //   11 fp32 products of M > 128 rows: 1 = the in-tree tiled GEMM instead of hipBLASLt
  m.def("set_variant", [](int64_t slot, int64_t v) {
    TORCH_CHECK(slot >= 0 && slot < 24, "variant slot");
    sl::g_variant[slot] = (int)v;
  });
  m.def("get_variant", [](int64_t slot) {
    TORCH_CHECK(slot >= 0 && slot < 24, "variant slot");
    return (int64_t)sl::g_variant[slot];
  });
  // compute dtype of the GEMM-shaped kernels (forward / data-gradient products): fp32 (exact
  // v_mfma_f32_*_f32) or bf16 (operands rounded to bf16, bf16 MFMA, fp32 accumulation);
  // parameters, optimizer state and the fused optimizer update stay fp32 either way
  m.def("set_compute_dtype", [](const std::string& d) {
    TORCH_CHECK(d == "fp32" || d == "bf16", "compute dtype fp32 | bf16");
    sl::g_bf16 = d == "bf16" ? 1 : 0;
  });
  m.def("get_compute_dtype", []() { return std::string(sl::g_bf16 ? "bf16" : "fp32"); });
  // gemm_nn_dgrad's split over the reduction: 0 = its own choice (default), else forced (sweeps)
  m.def("set_gemm_nn_splits", [](int s) { sl::g_nn_splits = s < 0 ? 0 : s; });
  m.def("set_gemm_nn_form", [](int wm) { sl::g_nn_wm = (wm == 2 || wm == 4) ? wm : 0; });
  m.def("set_gemm_nt_splits", [](int s) { sl::g_nt_splits = s < 0 ? 0 : s; });
  // hand-off stress test (csrc/handoff.hip, tests/test_handoff_gpu.py): G workgroups x R rounds
  // of the persistent kernels' publication primitive in `mode`; returns {mismatching words,
  // rounds completed by the slowest workgroup, error word, kernel ms, first mismatch [7]...}
  m.def("handoff_stress", [](int64_t G, int64_t P, int64_t R, int64_t nsrc, int64_t src_stride, int64_t mode,
                             double busy_us, double timeout_s) {
    sl::HoArgs a{};
    a.P = (int)P;
    a.R = (int)R;
    a.nsrc = (int)nsrc;
    a.src_stride = (int)src_stride;
    a.mode = (int)mode;
    const std::string why = sl::handoff_check(a, (int)G);
    TORCH_CHECK(why.empty(), "handoff_stress: ", why);
    int dev = 0, khz = 0;
    TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "device");
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    auto fo = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev);
    auto io = fo.dtype(at::kInt);
    at::Tensor D = at::zeros({G * P}, fo), S = at::zeros({G * sl::kHoScratchF4 * 4}, fo);
    at::Tensor cnt = at::zeros({2 * 8 * sl::kHoStride}, io), bad = at::zeros({G}, io), done = at::zeros({G}, io);
    at::Tensor first = at::zeros({8}, io), err = at::zeros({1}, io);
    a.D = D.data_ptr<float>();
    a.scratch = S.data_ptr<float>();
    a.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr<int>());
    a.bad = reinterpret_cast<unsigned*>(bad.data_ptr<int>());
    a.done = reinterpret_cast<unsigned*>(done.data_ptr<int>());
    a.first = reinterpret_cast<unsigned*>(first.data_ptr<int>());
    a.err = err.data_ptr<int>();
    a.timeout = (int64_t)(timeout_s * 1000.0 * khz);
    a.busy_ticks = (int)(busy_us * khz / 1000.0);
    const hipStream_t st = cur_stream();
    hipEvent_t e0, e1;
    TORCH_CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess, "events");
    TORCH_CHECK(hipEventRecord(e0, st) == hipSuccess, "event");
    check(sl::handoff_stress_launch(a, (int)G, st), "handoff_stress");
    TORCH_CHECK(hipEventRecord(e1, st) == hipSuccess, "event");
    TORCH_CHECK(hipEventSynchronize(e1) == hipSuccess, "handoff_stress sync");
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    const int64_t nbad = bad.to(at::kLong).sum().item<int64_t>();
    const int64_t rmin = done.min().item<int>();
    std::vector<int64_t> f(7);
    auto fc = first.cpu();
    for (int i = 0; i < 7; ++i) f[i] = (int64_t)(uint32_t)fc.data_ptr<int>()[i];
    return pybind11::make_tuple(nbad, rmin, err.item<int>(), (double)ms, f);
  });
  m.attr("arch") = "gfx950";
}
