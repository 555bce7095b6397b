// Vanilla persistent split epoch: every batch of a co-located Alice's vanilla epoch, her conv
// front and Bob's 3-layer tail, in ONE cooperative launch (one workgroup per CU).
//
// Reference: the vanilla hot loop (data_entities_vanilla.py:66-76): per batch, Alice's
// model1_sisa forward (Conv2d(1, 32, 3) -> ReLU -> MaxPool(2, 2) -> flatten, models.py:16-30),
// Bob's model2_sisa forward + CE (fc1 5408 -> 5000, ReLU, dropout 0.5, fc2 5000 -> 1000, ReLU,
// dropout 0.5, fc3 1000 -> 100, models.py:46-63), the distributed backward through both, and
// one SGD-momentum step of both sides (data_entities_vanilla.py:37-42).
//
// Why.  The launch-per-stage vanilla batch (csrc/split.cpp) is nine launches, 167 us on an
// MI355X: a 93 us SGD wgrad stream of all 32 M Bob parameters, a 25 us cut-gradient pass over
// W1 and seven 5-8 us latency-bound launches (profiles/r3e_vanilla_kernel_stats.csv).  Here
// fc2 / fc3 and the biases stay on-chip for the whole epoch (hybrid.hip's layout: fc2 tile W in
// LDS, its momentum in VGPRs), and per step only fc1 streams, twice: an UPDATE pass (W1 and its
// momentum read and written once, 432 MB) that also forms the cut gradient dx = dz1 W1_i from
// the old weights it already holds, and a FORWARD pass (W1 read once, 108 MB) of the next
// batch over the updated weights.  The two cannot merge: the next batch's activation depends
// on Alice's step, which needs the whole cut gradient of this one.
//
// Step i, workgroup w (G = 256; fc2 tile (ta, tb) = (w / NC, w % NC); conv job (c, g) =
// (w % 32, w / 32): channel c of the batch's images 2 g, 2 g + 1):
//   F, H, S, H2, B   Bob's head chain exactly as hybrid.hip (h1 from the forward partials, fc2
//                    partials, logits, softmax-CE, dz2, dz1 partials, W2's step in place)
//   U  dz1 of the workgroup's update run (column-major: one or two column blocks of 256
//      inputs, ~27 row blocks of 16 rows), b1's step by each row block's forward owner; per
//      16 x 256 tile: dW = dz1^T x_i (VALU), dx += dz1 W1_i (exact-fp32 MFMA on the old W the
//      lane holds: no LDS staging), SGD-momentum on W / buf, write-through stores.  At a column
//      block's end the run's dx partial -> DX[cb][slot] and one arrival on XD[cb].
//   C  conv job: its 2 x 169 cut-gradient entries (the column block partials in slot order),
//      the pool / ReLU backward (the argmax and value kept in VGPRs since the forward), the
//      10 conv gradients of (c, g) -> CWP, arrival on CW[c]; every job of channel c then sums
//      the 8 pairs' partials in order and applies the same SGD-momentum step (no owner, no
//      second hand-off), and runs the forward of batch i + 1 for (c, g) -> its activation
//      slot, seam X.
//   V  the forward pass of batch i + 1 (row-major runs, hybrid.hip's look-ahead product on
//      the updated tiles staged through LDS) -> LA partials, arrivals on R[rb].
// A prologue runs Alice's forward of batch 0 and the forward pass V of it.  Tiles written by
// one workgroup's update run are read by another's forward run: every fc1 store is write-
// through (sc1) and drained before the arrival that orders it, and every fc1 load is an sc1
// load (MI355X_MICROARCH.md, the valid-forms table row 1).  The activation slots are handed
// off the same way (sc1 stores by the conv jobs, sc1 loads after seam X): every load of
// handed-off bytes in this kernel is an sc1 load, as the row requires (plain loads of an sc1-
// stored payload read stale L1 lines: csrc/handoff.hip mode 2).  All sums run in a fixed order:
// a launch is deterministic and one launch of S steps is bitwise S one-step launches.
//
// REMOTE Alice (the <true> instantiation; BASELINE config 3, where 3 of 4
// Alices live on other GPUs; reference data_entities_vanilla.py:56-76 with split_nn.py:49-52's
// round-robin).  Her conv front runs in her process (csrc/split.cpp run_alice, unchanged) and
// this launch speaks the peer-mapped channel's protocol (csrc/ipc_p2p.h) in place of the C
// phase's conv jobs:
//   C_send  workgroup c < the message's chunks: wait every column block's cut-gradient
//           partials (XD), the ack of the message two generations back, then its 1,024 floats
//           of dx_i (the partials in slot order, as the conv jobs sum them) as system-scope
//           write-through stores into her slot over xGMI -> drain -> release -> flag = gen;
//   C_recv  (batch i + 1) every workgroup its 1 / G share of the [16][K1] activation slot:
//           poll the flags of the chunks it reads (relaxed system loads, then one acquire),
//           system-scope loads of her message, sc1 stores into the step's slot in the MFMA A
//           layout (padding rows zero), workgroup 0 the labels -> Yrem -> seam X; after seam X
//           the message's chunks are acked (every read of it has drained).
// So her messages, their sizes and their order are run_bob's: she cannot tell which executor
// served her, and the per-batch Bob path stays the fallback with no change on her side.
#include "vanilla.h"
#include "ipc_ar.h"
#include "persist.h"

#include <string>

namespace sl {

namespace {

using namespace persist;

__device__ __forceinline__ unsigned* va_cnt(const VaArgs& a, int i) { return a.cnt + i * kVaStride; }
__device__ __forceinline__ int va_seam(int seam, int shard) { return seam * 8 + shard; }
__device__ __forceinline__ int va_P(int b) { return kVaSeams * 8 + b; }
__device__ __forceinline__ int va_R(int rb) { return kVaSeams * 8 + kVaMaxNC + rb; }
__device__ __forceinline__ int va_XD(int cb) { return kVaSeams * 8 + kVaMaxNC + kVaMaxRB + cb; }
__device__ __forceinline__ int va_CW(int c) { return kVaSeams * 8 + kVaMaxNC + kVaMaxRB + kVaMaxCB + c; }
__device__ __forceinline__ int va_CX(int c) { return kVaSeams * 8 + kVaMaxNC + kVaMaxRB + kVaMaxCB + 32 + c; }

__device__ __forceinline__ bool va_spin(const VaArgs& a, const unsigned* p, unsigned tgt) {
  if (poll(p) >= tgt) return true;
  const uint64_t t0 = wall_clock64();
  while (poll(p) < tgt) {
    if (failed(a.err)) return false;
    __builtin_amdgcn_s_sleep(1);
    if ((int64_t)(wall_clock64() - t0) > a.timeout) {
      __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ void va_arrive(const VaArgs& a, int idx) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(va_cnt(a, idx), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool va_seam_wait(const VaArgs& a, int seam, unsigned mult, int* s_ok, const int* s_sn) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < 8) {
      const unsigned tg = mult * (unsigned)s_sn[seam * 8 + lane];
      if (tg > 0) ok = va_spin(a, va_cnt(a, va_seam(seam, lane)), tg);
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  asm volatile("" ::: "memory");   // no load of the handed-off bytes is hoisted above the wait
  return *s_ok != 0;
}

// wave 0's lanes [0, n) wait for counters idx0 + lane to reach tgt(lane); uniform result
template <typename F>
__device__ __forceinline__ bool va_wait_many(const VaArgs& a, int n, int* s_ok, F tgt_of) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < n) {
      int idx;
      const unsigned tg = tgt_of(lane, idx);
      if (tg > 0) ok = va_spin(a, va_cnt(a, idx), tg);
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  asm volatile("" ::: "memory");   // no load of the handed-off bytes is hoisted above the wait
  return *s_ok != 0;
}

// one lane: bounded wait until the channel flag / ack word *f reaches generation `want`
// (remote Alice); a timeout raises the launch's error word and the channel's
__device__ __forceinline__ bool va_pwait(const VaArgs& a, const uint32_t* f, uint32_t want) {
  if ((int32_t)(ipc_poll_flag(f) - want) >= 0) return true;
  const uint64_t t0 = wall_clock64();
  while ((int32_t)(ipc_poll_flag(f) - want) < 0) {
    if (failed(a.err)) return false;
    __builtin_amdgcn_s_sleep(1);
    if ((int64_t)(wall_clock64() - t0) > a.timeout) {
      __hip_atomic_fetch_or(a.err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ipc_fail(a.lk.err, a.lk.herr);
      return false;
    }
  }
  return true;
}

constexpr int kSt = 16;   // fc1 W / buf loads and stores: sc1 (write-through stores, L1-bypassing loads)
constexpr int kVaFwdRing = 6;   // forward-pass register ring depth (tiles; kVaFwdRing - 1 in flight)
constexpr int kVaFwdPre = 2;    // of them loaded early, under the seam-X wait (VGPR budget: 3 spill)
// seam X of a co-located Alice: her 32 x 8 conv jobs arrive on one counter per channel (8 each)
// and wave 0's 32 lanes poll them, instead of 8 shards of 32 arrivals.  Off: no faster (137.0
// vs 136.4 us, profiles/r6_vanilla_direct/seam_x_per_channel_ab.txt)
constexpr bool kVaSeamXByChannel = false;

// f(integral_constant<int, I>) for I in [B, E): compile-time ring and buffer indices in the
// unrolled tile loops
template <int B, int E, typename F>
__device__ __forceinline__ void va_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    va_static_for<B + 1, E>(f);
  }
}

// LDS carve (bytes)
constexpr int PW2 = 4 * kVaMaxWC4 + 1;
constexpr int PH = 4 * kVaMaxWC4 + 4;
constexpr int PD = kVaMaxWR + 1;
constexpr int OFF_W2 = 0;
constexpr int OFF_U = OFF_W2 + ((kVaMaxWR * PW2 * 4 + 15) & ~15);
// union, update-pass view: x_i column block [16][64] f32x4 (also the dx flush scratch), dz1 of
// the forward run's row blocks [kVaRuns][16 m][16] (b1's step)
constexpr int U_SA = 0;
constexpr int U_DZB = U_SA + 16 * 64 * 16;
constexpr int kUUpd = U_DZB + kVaRuns * 256 * 4;
// union, forward-pass view: the flush's last-row-block accumulators [8 waves][64] f32x4 at U_SA,
// the earlier row blocks' [kVaRuns - 1][8 waves][64] f32x4 behind them (no global round trip)
constexpr int U_ZP = U_SA + 8 * 64 * 16;
constexpr int kUFwd = U_ZP + (kVaRuns - 1) * 8 * 64 * 16;
// union, fc2 view
constexpr int U_SH1 = 0;
constexpr int U_SDZ2 = U_SH1 + 16 * PH * 4;
constexpr int U_RED = U_SDZ2 + ((16 * PD * 4 + 15) & ~15);
constexpr int U_SDL = U_RED + 16 * 32 * 16;
constexpr int U_SH2 = U_SDL + 16 * kVaMaxC * 4;
constexpr int U_SDZH = U_SH2 + 16 * 4 * 4;
constexpr int kUFc2 = U_SDZH + 16 * 4 * 4;
constexpr int kU0 = kUUpd > kUFc2 ? kUUpd : kUFc2;
constexpr int kU = kU0 > kUFwd ? kU0 : kUFwd;
constexpr int OFF_W3 = OFF_U + kU;                       // W3 columns {W, buf}[4][kVaMaxC]
constexpr int OFF_B3 = OFF_W3 + 2 * 4 * kVaMaxC * 4;     // b3 {W, buf}[kVaMaxC]
constexpr int OFF_B2 = OFF_B3 + 2 * kVaMaxC * 4;         // b2 {W, buf}[4] (+ pad)
constexpr int OFF_B1 = OFF_B2 + 64;                      // b1 {W, buf, -}[kVaRuns][16]
constexpr int OFF_DZ1 = OFF_B1 + kVaRuns * 3 * 16 * 4;   // dz1 of the update run [kVaMaxRun][16 m][16]
constexpr int OFF_IMG = OFF_DZ1 + kVaMaxRun * 256 * 4;   // images [2 parity][2][784] bytes
constexpr int OFF_CV = OFF_IMG + 2 * 2 * 784;            // conv channel {w[9], b, buf w[9], buf b} (+ pad)
constexpr int OFF_CRED = OFF_CV + 32 * 4;                // conv gradient reduction [8 waves][16]
constexpr int OFF_OK = OFF_CRED + 8 * 16 * 4;
constexpr int OFF_TABC = OFF_OK + 64;
constexpr int kVaLds = OFF_TABC + (32 + kVaRuns + kVaSeams * 8 + kVaMaxCB) * 4 + 16;
static_assert(kVaLds <= 160 * 1024, "LDS");
static_assert(kVaThreads / 64 * 10 * 256 >= kVaMaxWR * 4 * kVaMaxWC4, "10 W2 16 x 16 blocks per wave");

}  // namespace

#define VA_IDX()                                                           \
  int tid_l_ = threadIdx.x;                                                \
  asm volatile("" : "+v"(tid_l_));                                         \
  const int tid = tid_l_, r = tid >> 6, lane = tid & 63, li = lane & 15, lq = lane >> 4; \
  (void)r; (void)lane; (void)li; (void)lq

// phase stamps of every workgroup for steps tall_step .. (scripts/vanilla_trace.py)
#define VA_MARK(k)                                                                             \
  do {                                                                                         \
    if (threadIdx.x == 0 && a.tall != nullptr && i >= a.tall_step && i < a.tall_step + a.tall_n) \
      a.tall[((int64_t)(i - a.tall_step) * G + w) * 16 + (k)] = (int64_t)wall_clock64();     \
  } while (0)

// REM: the Alice is remote (the channel phases above in place of the conv jobs)
template <bool REM>
__global__ void __launch_bounds__(kVaThreads) vanilla_epoch_kernel(VaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sw2 = reinterpret_cast<float*>(smem + OFF_W2);
  f32x4* sa = reinterpret_cast<f32x4*>(smem + OFF_U + U_SA);
  f32x4* szp = reinterpret_cast<f32x4*>(smem + OFF_U + U_ZP);
  float* sdzb = reinterpret_cast<float*>(smem + OFF_U + U_DZB);
  float* sh1 = reinterpret_cast<float*>(smem + OFF_U + U_SH1);
  float* sdz2 = reinterpret_cast<float*>(smem + OFF_U + U_SDZ2);
  f32x4* red = reinterpret_cast<f32x4*>(smem + OFF_U + U_RED);
  float* sdl = reinterpret_cast<float*>(smem + OFF_U + U_SDL);
  float* sh2 = reinterpret_cast<float*>(smem + OFF_U + U_SH2);
  float* sdzh = reinterpret_cast<float*>(smem + OFF_U + U_SDZH);
  float* sW3 = reinterpret_cast<float*>(smem + OFF_W3);
  float* sb3 = reinterpret_cast<float*>(smem + OFF_B3);
  float* sb2 = reinterpret_cast<float*>(smem + OFF_B2);
  float* sb1 = reinterpret_cast<float*>(smem + OFF_B1);
  float* sdz1 = reinterpret_cast<float*>(smem + OFF_DZ1);
  uint8_t* simg = reinterpret_cast<uint8_t*>(smem + OFF_IMG);
  float* scv = reinterpret_cast<float*>(smem + OFF_CV);
  float* scred = reinterpret_cast<float*>(smem + OFF_CRED);
  int* s_ok = reinterpret_cast<int*>(smem + OFF_OK);
  int* s_fns = reinterpret_cast<int*>(smem + OFF_TABC);   // [32]: forward slots of row block rlo + j
  int* s_slot = s_fns + 32;                                // [kVaRuns]: w - first forward toucher
  int* s_sn = s_slot + kVaRuns;                            // [kVaSeams * 8]
  int* s_dxs = s_sn + kVaSeams * 8;                        // [kVaMaxCB]: this run's dx slot per column block
  constexpr int MC = kVaMaxC;
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};

  const int w = blockIdx.x;
  const int M = a.M, N1 = a.N1, K1 = a.K1, N2 = a.N2, C = a.C, C4 = a.C4, G = a.G, NC = a.NC;
  const int ncb = a.ncb, nrb = a.nrb;
  const int ta = w / NC, tb = w - (w / NC) * NC;
  const int Q2 = N2 >> 2, Q4 = N1 >> 2;
  const int r0 = 4 * (ta * Q2 / kVaNR), WR = 4 * ((ta + 1) * Q2 / kVaNR) - r0;
  const int q0 = tb * Q4 / NC, WC4 = (tb + 1) * Q4 / NC - q0;
  const int c0 = 4 * q0, WC = 4 * WC4;
  const bool head = w < a.HW;
  // forward-pass tile run (row-major) [t_begin, t_end), row blocks rbA .. rbA + nruns - 1
  const int t_begin = a.tab[w], t_end = a.tab[w + 1];
  const int nt = t_end - t_begin;
  const int rbA = nt > 0 ? t_begin / ncb : 0;
  const int nruns = nt > 0 ? (t_end - 1) / ncb - rbA + 1 : 0;
  // update-pass tile run [u_begin, u_begin + unt) of the row band [u_rb0, u_rb0 + u_nb), walked
  // column-major (tile v: column block v / u_nb, row block u_rb0 + v % u_nb)
  const int u_begin = a.tab[a.oUW + 4 * w], unt = a.tab[a.oUW + 4 * w + 1] - u_begin;
  const int u_rb0 = a.tab[a.oUW + 4 * w + 2], u_nb = a.tab[a.oUW + 4 * w + 3];
  // conv job: channel cc, images 2 cg, 2 cg + 1
  const int cc = w & 31, cg = w >> 5;
  const __amdgpu_buffer_rsrc_t rHB = rs_of(a.HB);
  const int bLA = 4 * a.oLA, bH1 = 4 * a.oH1, bFP = 4 * a.oFP, bLP = 4 * a.oLP, bDL = 4 * a.oDL, bDZ = 4 * a.oDZ,
            bDP = 4 * a.oDP, bDX = 4 * a.oDX, bCW = 4 * a.oCWP;
  const __amdgpu_buffer_rsrc_t rX = rs_of(a.Xr);
  const __amdgpu_buffer_rsrc_t rW1 = rs_of(a.L1.W), rM1 = rs_of(a.L1.m);

  // ---- resident state: the W2 tile (LDS), its momentum (VGPRs), head columns, biases, conv channel
  f32x4 m2[10];
  {
    VA_IDX();
    for (int e = tid; e < kVaMaxWR * PW2; e += kVaThreads) sw2[e] = 0.f;
    __syncthreads();
    for (int e = tid; e < WR * WC4; e += kVaThreads) {
      const int n = e / WC4, q = e - n * WC4;
      const f32x4 wv = *reinterpret_cast<const f32x4*>(a.L2.W + (int64_t)(r0 + n) * N1 + c0 + 4 * q);
#pragma unroll
      for (int k = 0; k < 4; ++k) sw2[n * PW2 + 4 * q + k] = wv[k];
    }
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int b = r + 8 * u, bn = b / 10, bk = b - (b / 10) * 10;
      m2[u] = zv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * bn + 4 * lq + j, k = 16 * bk + li;
        if (n < WR && k < WC) m2[u][j] = a.L2.m[(int64_t)(r0 + n) * N1 + c0 + k];
      }
    }
    if (head && tid < 4 * MC) {
      const int ii = tid / MC, c = tid - ii * MC;
      const int n = 4 * w + ii;
      const bool ok = c < C;
      const int64_t off = (int64_t)c * N2 + n;
      sW3[(0 * 4 + ii) * MC + c] = ok ? a.L3.W[off] : 0.f;
      sW3[(1 * 4 + ii) * MC + c] = ok ? a.L3.m[off] : 0.f;
    }
    if (tid < MC) {
      const bool ok = tid < C;
      sb3[tid] = ok ? a.L3.b[tid] : 0.f;
      sb3[MC + tid] = ok ? a.L3.mb[tid] : 0.f;
    }
    if (head && tid < 4) {
      const int n = 4 * w + tid;
      sb2[tid] = a.L2.b[n];
      sb2[4 + tid] = a.L2.mb[n];
    }
    if (tid < 32) {
      const int rb = (c0 >> 4) + tid;
      s_fns[tid] = rb <= ((c0 + WC - 1) >> 4) && rb < nrb ? a.tab[G + 1 + nrb + rb] : 0;
    }
    if (tid < kVaRuns) s_slot[tid] = tid < nruns ? w - a.tab[G + 1 + rbA + tid] : -1;
    if (tid < kVaSeams * 8) s_sn[tid] = a.shard_n[tid];
    if (tid < kVaMaxCB) s_dxs[tid] = tid < ncb ? a.tab[a.oUS + w * ncb + tid] : -1;
    if (tid < 16 * kVaRuns) {
      const int k = tid >> 4, j = tid & 15;
      const int rb = rbA + k, n = 16 * rb + j;
      const bool own = k < nruns && a.tab[G + 1 + rb] == w && n < N1;
      sb1[(k * 3 + 0) * 16 + j] = own ? a.L1.b[n] : 0.f;
      sb1[(k * 3 + 1) * 16 + j] = own ? a.L1.mb[n] : 0.f;
      sb1[(k * 3 + 2) * 16 + j] = 0.f;
    }
    if (!REM && tid < 20) {
      // {w[9], b, buf w[9], buf b} of channel cc
      const int j = tid < 10 ? tid : tid - 10;
      const float* src = tid < 10 ? (j < 9 ? a.cw + cc * 9 + j : a.cb + cc) : (j < 9 ? a.cmw + cc * 9 + j : a.cmb + cc);
      scv[tid] = *src;
    }
  }

  // ---------------------------------------------------------------- Alice's conv job
  // the step's images 2 cg, 2 cg + 1 as 196 words each (thread < 392); zero for padding rows
  auto img_word = [&](int step) -> uint32_t {
    VA_IDX();
    uint32_t v = 0;
    if (tid < 392 && step < a.S) {
      const int bl = tid / 196, wd = tid - (tid / 196) * 196;
      const int m = 2 * cg + bl;
      const int64_t src = m < M ? a.rows[(int64_t)step * M + m] : -1;
      if (src >= 0) v = reinterpret_cast<const uint32_t*>(a.img + src * 784)[wd];
    }
    return v;
  };
  auto img_put = [&](int par, uint32_t v) {
    VA_IDX();
    if (tid < 392) reinterpret_cast<uint32_t*>(simg + par * 1568)[tid] = v;
  };
  // pooled output (image bl, position p) of channel cc over image buffer par: conv.hip's
  // conv_pool_at arithmetic (first max in torch order, then ReLU)
  auto conv_at = [&](int par, int bl, int p, float& y, int& arg) {
    const uint8_t* im = simg + par * 1568 + bl * 784;
    const int ph = p / 13, pw = p - (p / 13) * 13;
    float patch[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) patch[i][j] = (float)im[(2 * ph + i) * 28 + 2 * pw + j];
    float best = 0.f;
    arg = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float acc = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) acc = fmaf(scv[kh * 3 + kw], patch[dy + kh][dx + kw], acc);
        acc += scv[9];
        const int pos = dy * 2 + dx;
        if (pos == 0 || acc > best) {
          best = acc;
          arg = pos;
        }
      }
    y = fmaxf(best, 0.f);
  };
  // activation slot layout [K1 / 16][16 m][16 k] per step: the forward pass's MFMA A operand
  // (row m = lane % 16, four consecutive k) is then one contiguous 1 KB per wave load (row-major
  // [16][K1], 16 rows x 64 B per load, cost ~7 us of the 32 us forward pass)
  auto xoff = [&](int step, int m, int k) { return ((step * (K1 >> 4) + (k >> 4)) * 16 + m) * 16 + (k & 15); };
  // forward of step `step` for this job -> activation slot `step`; keeps (y, arg) for the backward
  float cy = 0.f;
  int carg = 0;
  auto conv_fwd = [&](int step) {
    VA_IDX();
    if (tid < 338) {
      const int bl = tid / 169, p = tid - (tid / 169) * 169;
      const int m = 2 * cg + bl;
      const bool valid = m < M && a.rows[(int64_t)step * M + m] >= 0;
      float y = 0.f;
      int arg = 0;
      if (valid) conv_at(step & 1, bl, p, y, arg);
      cy = y;
      carg = arg;
      hst1(rX, xoff(step, m, cc * 169 + p) * 4, y);
    }
  };

  // ---------------------------------------------------------------- fc1 forward pass
  f32x4 sp[2][2], sm[2][2];
  // W1 tile t straight in the MFMA B layout (no LDS staging): lane (li, lq) of wave r holds row
  // 16 rb + li, columns 256 cb + 16 (r + 8 h) + 4 lq .. + 3 -- the operand the wave's MFMAs take
  // (a wave's load: 16 rows x 64 B; two waves share each 128-B line)
  auto load_w = [&](int t, f32x4 (&p)[2]) {
    VA_IDX();
    const int rb = t / ncb, cb = t - (t / ncb) * ncb;
    const int n = 16 * rb + li;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = cb * 256 + 16 * (r + 8 * h) + 4 * lq;
      p[h] = (n < N1 && k < K1)
                 ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rW1, (n * K1 + k) * 4, 0, kSt))
                 : zv;
    }
  };
  auto load_xv = [&](int step, int t, f32x4 (&xv)[2]) {
    VA_IDX();
    const int cb = t - (t / ncb) * ncb;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = cb * 256 + 16 * (r + 8 * h) + 4 * lq;
      xv[h] = k < K1 ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rX, xoff(step, li, k) * 4, 0, kSt)) : zv;
    }
  };
  f32x4 zlast = zv;
  // a finished row block's per-wave accumulator -> LDS (read by this workgroup's flush only)
  auto zp_store = [&](int k, f32x4 z) {
    VA_IDX();
    szp[(k * 8 + r) * 64 + lane] = z;
  };
  // The forward pass keeps kVaFwdRing - 1 tiles of W (sc1 loads: tiles another workgroup's
  // update run just wrote) and x in flight in a register ring, every load issued after the
  // seam-X wait that orders it (all of the step's fc1 stores drained before any conv job
  // arrived, docs/PERF.md round 6); ring slot = tile index % kVaFwdRing, compile-time in the
  // unrolled loop.  Both operands are loaded in their MFMA layouts, so every wave streams its
  // own k-slice of each tile with no LDS staging and no workgroup barrier per tile (the staged
  // form: a 16 KB LDS round trip and a barrier per tile, 4.3 TB/s).  Same products in the same
  // order at every depth and in both forms: the form and the depth change timing only.
  // The ring's first W tiles are loaded early (fwd_prefetch), under the seam-X wait: once every
  // update run of the step has arrived (XD), W no longer waits for anything, only x does.
  constexpr int kPre = kVaFwdPre;
  f32x4 wpre[kPre > 0 ? kPre : 1][2];
  auto fwd_prefetch = [&]() {
#pragma unroll
    for (int d = 0; d < kPre; ++d)
      if (d < nt) load_w(t_begin + d, wpre[d]);
  };
  // every update run of step i has stored and drained its tiles (the W the forward pass reads)
  auto wait_all_xd = [&](int i) {
    return va_wait_many(a, ncb, s_ok, [&](int l, int& idx) {
      idx = va_XD(l);
      return (unsigned)(i + 1) * (unsigned)a.tab[a.oU + l];
    });
  };
  auto fwd_pass = [&](int step) {
    if (nt <= 0) return;
    constexpr int D = kVaFwdRing;
    static_assert(D >= 2 && D % 2 == 0, "ring depth: even, >= 2");
    f32x4 wr[D][2], xr[D][2];
#pragma unroll
    for (int d = 0; d < D - 1; ++d)
      if (d < nt) {
        if (d < kPre) {
          wr[d][0] = wpre[d][0];
          wr[d][1] = wpre[d][1];
        } else {
          load_w(t_begin + d, wr[d]);
        }
        load_xv(step, t_begin + d, xr[d]);
      }
    f32x4 z = zv;
    int kz = 0;
    auto tile = [&](auto cur_c, int j) {
      constexpr int cur = decltype(cur_c)::value, nx = (cur + D - 1) % D;
      const int t = t_begin + j;
      const int rb = t / ncb;
      const int kr = rb - rbA;
      if (kr != kz) {
        zp_store(kz, z);
        z = zv;
        kz = kr;
      }
      if (j + D - 1 < nt) {
        load_w(t + D - 1, wr[nx]);
        load_xv(step, t + D - 1, xr[nx]);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 4; ++c) z = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[cur][h][c], wr[cur][h][c], z, 0, 0, 0);
    };
    int j = 0;
    for (; j + D - 1 < nt; j += D) va_static_for<0, D>([&](auto dc) { tile(dc, j + decltype(dc)::value); });
    va_static_for<0, D - 1>([&](auto dc) {
      if (j + decltype(dc)::value < nt) tile(dc, j + decltype(dc)::value);
    });
    zlast = z;
  };
  // the run's forward partials for step so (hybrid.hip's flush): each row block's partial (the
  // 8 waves' accumulators in order, + b1 by its first workgroup) -> LA, one arrival on R[rb]
  auto flush = [&](int so) {
    const int par = so & 1;
    {
      VA_IDX();
      __syncthreads();
      sa[r * 64 + lane] = zlast;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    {
      VA_IDX();
      for (int e = tid; e < nruns * 64; e += kVaThreads) {
        const int k = e >> 6, nn = (e >> 2) & 15, mg = e & 3;
        const int rb = rbA + k, slot = s_slot[k], n = 16 * rb + nn;
        f32x4 parts[8];
        if (k == nruns - 1) {
#pragma unroll
          for (int ww = 0; ww < 8; ++ww) parts[ww] = sa[ww * 64 + 16 * mg + nn];
        } else {
#pragma unroll
          for (int ww = 0; ww < 8; ++ww) parts[ww] = szp[(k * 8 + ww) * 64 + 16 * mg + nn];
        }
        f32x4 v = parts[0];
#pragma unroll
        for (int ww = 1; ww < 8; ++ww) v += parts[ww];
        if (slot == 0) v += sb1[(k * 3) * 16 + nn];
        if (n < N1) hst4(rHB, bLA + (((par * nrb + rb) * kVaSlots + slot) * 256 + nn * 16 + 4 * mg) * 4, v);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < (unsigned)nruns)
      __hip_atomic_fetch_add(va_cnt(a, va_R(rbA + threadIdx.x)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // ---------------------------------------------------------------- fc1 update pass
  // tile t (column-major): wave r = (row half rh, column quarter cq), lane (li, lq): rows
  // 16 rb + 8 rh + lq + 4 s (s = 0, 1), columns 256 cb + 64 cq + 4 li .. + 3
  auto load_u = [&](int t, f32x4 (&p)[2], f32x4 (&mm)[2]) {
    VA_IDX();
    const int rh = r >> 2, cq = r & 3;
    const int cb = t / u_nb, rb = u_rb0 + t - (t / u_nb) * u_nb;
    const int k = cb * 256 + 64 * cq + 4 * li;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int n = 16 * rb + 8 * rh + lq + 4 * s;
      const bool act = n < N1 && k < K1;
      const int boff = (n * K1 + k) * 4;
      p[s] = act ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rW1, boff, 0, kSt)) : zv;
      mm[s] = act ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rM1, boff, 0, kSt)) : zv;
    }
  };
  auto stage_x = [&](int cb, int step) {
    VA_IDX();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * kVaThreads;
      const int m = e >> 6, k = cb * 256 + 4 * (e & 63);
      sa[e] = k < K1 ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rX, xoff(step, m, k) * 4, 0, kSt)) : zv;
    }
  };
  f32x4 dacc[4];
  // the run's dx partial of column block cb -> DX[cb][slot], one arrival on XD[cb]
  auto flush_dx = [&](int cb) {
    __syncthreads();
    {
      VA_IDX();
      const int rh = r >> 2, cq = r & 3;
      if (rh == 1) {
#pragma unroll
        for (int c = 0; c < 4; ++c) sa[(cq * 4 + c) * 64 + lane] = dacc[c];
      }
    }
    __syncthreads();
    {
      VA_IDX();
      const int rh = r >> 2, cq = r & 3;
      if (rh == 0) {
        const int slot = s_dxs[cb];
#pragma unroll
        for (int c = 0; c < 4; ++c) dacc[c] += sa[(cq * 4 + c) * 64 + lane];
        const int k = 64 * cq + 4 * li;
        if (cb * 256 + k < K1) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const f32x4 v = {dacc[0][jj], dacc[1][jj], dacc[2][jj], dacc[3][jj]};
            hst4(rHB, bDX + (((cb * kVaDxSlots + slot) * 16 + 4 * lq + jj) * 256 + k) * 4, v);
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) dacc[c] = zv;
    va_arrive(a, va_XD(cb));
  };
  auto upd_pass = [&](int step, float ss, float ib) {
    if (unt <= 0) return;
    int ccb = u_begin / u_nb;
    stage_x(ccb, step);
#pragma unroll
    for (int c = 0; c < 4; ++c) dacc[c] = zv;
    __syncthreads();
    auto tile = [&](auto cur_c, int j) {
      constexpr int cur = decltype(cur_c)::value, nb = cur ^ 1;
      const int t = u_begin + j;
      const int cb = t / u_nb, rb = u_rb0 + t - (t / u_nb) * u_nb;
      if (cb != ccb) {   // uniform: the run enters its next column block
        flush_dx(ccb);
        ccb = cb;
        stage_x(cb, step);
        __syncthreads();
      }
      if (j + 1 < unt) load_u(t + 1, sp[nb], sm[nb]);
      VA_IDX();
      const int rh = r >> 2, cq = r & 3;
      const float* dz = sdz1 + j * 256;   // [16 m][16 rows]
      const int k = cb * 256 + 64 * cq + 4 * li;
      f32x4 g0 = zv, g1 = zv;
#pragma unroll 4
      for (int m = 0; m < 16; ++m) {
        const f32x4 xm = sa[m * 64 + 16 * cq + li];
        g0 += dz[m * 16 + 8 * rh + lq] * xm;
        g1 += dz[m * 16 + 8 * rh + lq + 4] * xm;
      }
      // cut gradient from the old tile: dx[m][k] += sum_n dz1[m][n] W1_i[n][k]; MFMA c takes
      // component c of the lane's float4 (columns 4 li + c), K = the 4 rows lq (+ 4 s)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float av = dz[li * 16 + 8 * rh + 4 * s + lq];
#pragma unroll
        for (int c = 0; c < 4; ++c) dacc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sp[cur][s][c], dacc[c], 0, 0, 0);
      }
      const int n0 = 16 * rb + 8 * rh + lq;
      const bool kin = k < K1;
      f32x4 dummy = zv;
      if (kin && n0 < N1) {
        res_update4<false>(a.o, ss, ib, sp[cur][0], g0, sm[cur][0], dummy);
        const int boff = (n0 * K1 + k) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, sp[cur][0]), rW1, boff, 0, kSt);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, sm[cur][0]), rM1, boff, 0, kSt);
      }
      if (kin && n0 + 4 < N1) {
        res_update4<false>(a.o, ss, ib, sp[cur][1], g1, sm[cur][1], dummy);
        const int boff = ((n0 + 4) * K1 + k) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, sp[cur][1]), rW1, boff, 0, kSt);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, sm[cur][1]), rM1, boff, 0, kSt);
      }
    };
    int j = 0;
    for (; j + 1 < unt; j += 2) {
      tile(std::integral_constant<int, 0>{}, j);
      tile(std::integral_constant<int, 1>{}, j + 1);
    }
    if (j < unt) tile(std::integral_constant<int, 0>{}, j);
    flush_dx(ccb);
  };

  // ---------------------------------------------------------------- remote Alice (REM)
  auto rows_of = [&](int s) { return (int)a.adam[4 * s]; };
  // her activation message of step s -> the step's slot (all 16 rows, padding rows zero), the
  // labels -> Yrem (workgroup 0); false when a wait gave up
  auto recv_act = [&](int s) -> bool {
    const int Ms = rows_of(s);
    const uint32_t rg = a.lk.rgen0 + 1u + (uint32_t)s;
    const int par = (int)(rg & 1u);
    const int K4 = K1 >> 2, NQ = 16 * K4;   // float4 groups of a row / of the slot
    const int q0 = (int)((int64_t)w * NQ / G), q1 = (int)((int64_t)(w + 1) * NQ / G);
    const int qm = Ms * K4;                  // float4 groups the message carries
    const int qe = q1 < qm ? q1 : qm;
    const int ca0 = 4 * q0 / kIpcChunk, na = qe > q0 ? (4 * qe - 1) / kIpcChunk - ca0 + 1 : 0;
    const int fl = Ms * K1;                  // the labels' first word
    const int cl0 = fl / kIpcChunk, nl = w == 0 ? (fl + 2 * Ms - 1) / kIpcChunk - cl0 + 1 : 0;
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      int c = -1;
      if (lane < na) c = ca0 + lane;
      else if (lane >= 32 && lane - 32 < nl) c = cl0 + lane - 32;
      bool ok = true;
      if (c >= 0) ok = va_pwait(a, a.lk.rflag[par] + c, rg);
      ok = __all(ok);
      ipc_acquire();
      if (lane == 0) *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (*s_ok == 0) return false;
    const __amdgpu_buffer_rsrc_t rR = ipc_rsrc(a.lk.rdata[par]);
    for (int q = q0 + (int)threadIdx.x; q < q1; q += kVaThreads) {
      const int m = q / K4, k = 4 * (q - m * K4);
      const f32x4 v = q < qm ? __builtin_bit_cast(f32x4, ipc_ld4(rR, 4 * (int64_t)q)) : zv;
      hst4(rX, xoff(s, m, k) * 4, v);
    }
    if (w == 0 && (int)threadIdx.x < M) {
      const int m = threadIdx.x;
      uint32_t lo = 0xffffff9cu, hi = 0xffffffffu;   // -100: a padding row, ignored
      if (m < Ms) {
        lo = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rR, (fl + 2 * m) * 4, 0, 17);
        hi = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rR, (fl + 2 * m + 1) * 4, 0, 17);
      }
      const __amdgpu_buffer_rsrc_t rY = rs_of(a.Yrem);
      hst1(rY, (s * M + m) * 8, __builtin_bit_cast(float, lo));
      hst1(rY, (s * M + m) * 8 + 4, __builtin_bit_cast(float, hi));
    }
    return true;
  };
  // after seam X every read of step s's message has drained: ack its chunks
  auto ack_act = [&](int s) {
    if (threadIdx.x == 0) {
      const int Ms = rows_of(s);
      const uint32_t rg = a.lk.rgen0 + 1u + (uint32_t)s;
      const int par = (int)(rg & 1u);
      const int nch = (((Ms * K1 + 2 * Ms + 3) & ~3) + kIpcChunk - 1) / kIpcChunk;
      for (int c = w; c < nch; c += G) ipc_raise_flag(a.lk.rack[par] + c, rg, 0);
    }
  };
  // the cut gradient of step i -> her slot (workgroup c: chunk c, 1,024 floats); false when a
  // wait gave up
  auto send_dx = [&](int i) -> bool {
    const int len = rows_of(i) * K1;
    const int nch = (len + kIpcChunk - 1) / kIpcChunk;
    if (w >= nch) return true;
    if (!va_wait_many(a, ncb, s_ok, [&](int l, int& idx) {
          idx = va_XD(l);
          return (unsigned)(i + 1) * (unsigned)a.tab[a.oU + l];
        }))
      return false;
    const uint32_t sg = a.lk.sgen0 + 1u + (uint32_t)i;
    const int par = (int)(sg & 1u);
    const int prev = i >= 2 ? (rows_of(i - 2) * K1 + kIpcChunk - 1) / kIpcChunk : a.lk.sprev[i];
    const __amdgpu_buffer_rsrc_t rS = ipc_rsrc(a.lk.sdata[par]);
    for (int c = w; c < nch; c += G) {
      if (threadIdx.x == 0) {
        // chunks beyond the message two generations back wait on its chunk 0 (ipc_p2p.hip)
        const bool ok = prev == 0 || va_pwait(a, a.lk.sack[par] + (c < prev ? c : 0), sg - 2u);
        ipc_acquire();
        *s_ok = ok ? 1 : 0;
      }
      __syncthreads();
      if (*s_ok == 0) return false;
      const int e = c * kIpcChunk + 4 * (int)threadIdx.x;
      if ((int)threadIdx.x < kIpcThreads && e < len) {
        const int m = e / K1, k = e - m * K1, cb = k >> 8, kk = k & 255;
        const int ns = a.tab[a.oU + cb];
        f32x4 parts[kVaDxSlots];
#pragma unroll
        for (int sl = 0; sl < kVaDxSlots; ++sl)
          parts[sl] = sl < ns ? hld4(rHB, bDX + (((cb * kVaDxSlots + sl) * 16 + m) * 256 + kk) * 4) : zv;
        f32x4 v = parts[0];
#pragma unroll
        for (int sl = 1; sl < kVaDxSlots; ++sl) v += parts[sl];
        ipc_st4(rS, e, __builtin_bit_cast(float4, v));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) ipc_raise_flag(a.lk.sflag[par] + c, sg);
      __syncthreads();   // s_ok is rewritten by the next chunk
    }
    return true;
  };

  // seam X: every activation of the next batch published (arrive, `between`, then wait);
  // REM: every workgroup's share of her message (8 shards), co-located: per channel (kVaSeamXByChannel)
  auto seam_x = [&](unsigned mult, auto between) -> bool {
    if (!REM && kVaSeamXByChannel) va_arrive(a, va_CX(cc));
    else va_arrive(a, va_seam(4, w & 7));
    if (!between()) return false;
    if (!REM && kVaSeamXByChannel)
      return va_wait_many(a, 32, s_ok, [&](int l, int& idx) {
        idx = va_CX(l);
        return mult * 8u;
      });
    return va_seam_wait(a, 4, mult, s_ok, s_sn);
  };

  // ---- prologue: Alice's forward of batch 0 (REM: her message of it), then the forward pass
  if constexpr (REM) {
    if (!recv_act(0)) goto done;
  } else {
    img_put(0, img_word(0));
    __syncthreads();
    conv_fwd(0);
  }
  if (!seam_x(1u, [] { return true; })) goto done;
  if constexpr (REM) ack_act(0);
  fwd_prefetch();
  fwd_pass(0);
  flush(0);

  for (int i = 0; i < a.S; ++i) {
    const int par = i & 1;
    const bool more = i + 1 < a.S;
    const uint32_t sd2 = a.seeds[4 * i + 2], sd3 = a.seeds[4 * i + 3];
    const SlOpt o = a.o;
    float ss = 0.f, ib = 0.f;
    asm volatile("" : "+v"(ss), "+v"(ib));
    VA_MARK(0);
    // the next batch's images, in flight across the step (written to LDS in the conv phase)
    const uint32_t pimg = (!REM && more) ? img_word(i + 1) : 0u;

    // ================= F: h1 slice, the tile's fc2 partial
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      const int rlo = c0 >> 4, rhi = (c0 + WC - 1) >> 4;
      bool ok = true;
      if (rlo + lane <= rhi) {
        const int rb = rlo + lane;
        const unsigned tg = i == a.fault_step ? 0xffffffffu : (unsigned)(i + 1) * (unsigned)s_fns[lane];
        ok = va_spin(a, va_cnt(a, va_R(rb)), tg);
      }
      ok = __all(ok);
      if (lane == 0) *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (*s_ok == 0) break;
    VA_MARK(1);
    {
      VA_IDX();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = tid + u * kVaThreads;
        const int kc = e >> 2, mg = e & 3;
        if (kc < 4 * kVaMaxWC4) {
          f32x4 v = zv;
          if (kc < WC) {
            const int n = c0 + kc, rb = n >> 4, nn = n & 15;
            const int ns = s_fns[rb - (c0 >> 4)];
            f32x4 parts[kVaSlots];
#pragma unroll
            for (int sl = 0; sl < kVaSlots; ++sl)
              parts[sl] = sl < ns ? hld4(rHB, bLA + (((par * nrb + rb) * kVaSlots + sl) * 256 + nn * 16 + 4 * mg) * 4) : zv;
            v = parts[0];
#pragma unroll
            for (int sl = 1; sl < kVaSlots; ++sl) v += parts[sl];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int m = 4 * mg + j;
              v[j] = m < M ? drop_relu(v[j], a.seeds[4 * i], a.seeds[4 * i + 1], m, n, a.thr1, a.dsc1) : 0.f;
            }
            if (ta == 0) hst4(rHB, bH1 + ((par * N1 + n) * 16 + 4 * mg) * 4, v);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) sh1[(4 * mg + j) * PH + kc] = v[j];
        }
      }
    }
    __syncthreads();
    {
      VA_IDX();
      if (16 * r < WR) {
        f32x4 acc0 = zv, acc1 = zv;
        const float* pa = sh1 + li * PH + lq;
        const float* pb = sw2 + (16 * r + li) * PW2 + lq;
#pragma unroll
        for (int kk = 0; kk < kVaMaxWC4; kk += 2) {
          if (kk < WC4) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * kk], pb[4 * kk], acc0, 0, 0, 0);
          if (kk + 1 < WC4) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * kk + 4], pb[4 * kk + 4], acc1, 0, 0, 0);
        }
        const f32x4 acc = acc0 + acc1;
        const int n = 16 * r + li;
        if (n < WR) hst4(rHB, bFP + (((par * NC + tb) * N2 + r0 + n) * 16 + 4 * lq) * 4, acc);
      }
    }
    va_arrive(a, va_seam(0, w & 7));

    VA_MARK(2);
    // ================= H: the head rows' fc2 sums, h2, logit partials
    if (head) {
      if (!va_seam_wait(a, 0, (unsigned)(i + 1), s_ok, s_sn)) break;
      {
        VA_IDX();
        const int cq = tid >> 4, ii = (tid >> 2) & 3, mg = tid & 3;
        red[tid] = cq < NC ? hld4(rHB, bFP + (((par * NC + cq) * N2 + 4 * w + ii) * 16 + 4 * mg) * 4) : zv;
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        VA_IDX();
        const int m = tid >> 2, ii = tid & 3;
        float pv = red[ii * 4 + (m >> 2)][m & 3];
#pragma unroll
        for (int cq = 1; cq < kVaMaxNC; ++cq) pv += red[cq * 16 + ii * 4 + (m >> 2)][m & 3];
        const int n = 4 * w + ii;
        sh2[m * 4 + ii] = m < M ? drop_relu(pv + sb2[ii], sd2, sd3, m, n, a.thr2, a.dsc2) : 0.f;
      }
      __syncthreads();
      {
        VA_IDX();
        const int nc4 = C4 >> 2;
        if (tid < 16 * nc4) {
          const int m = tid / nc4, c = 4 * (tid - m * nc4);
          if (m < M) {
            f32x4 v = zv;
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) v += sh2[m * 4 + ii] * *reinterpret_cast<const f32x4*>(sW3 + ii * MC + c);
            hst4(rHB, bLP + (((par * a.HW + w) * 16 + m) * C4 + c) * 4, v);
          }
        }
      }
      va_arrive(a, va_seam(1, w & 7));
    }

    // ================= S: row m's logits, softmax-CE, dlogits (workgroups m < M)
    if (w < M) {
      if (!va_seam_wait(a, 1, (unsigned)(i + 1), s_ok, s_sn)) break;
      const int m = w;
      const int nc4 = C4 >> 2;
      constexpr int NG = kVaThreads / 32;
      {
        VA_IDX();
        const int c4 = tid & 31, gq = tid >> 5;
        f32x4 v = zv;
        if (c4 < nc4) {
          f32x4 parts[256 / NG];
#pragma unroll
          for (int k = 0; k < 256 / NG; ++k) {
            const int src = gq + NG * k;
            parts[k] = src < a.HW ? hld4(rHB, bLP + (((par * a.HW + src) * 16 + m) * C4 + 4 * c4) * 4) : zv;
          }
#pragma unroll
          for (int k = 0; k < 256 / NG; ++k) v += parts[k];
        }
        red[gq * 32 + c4] = v;
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        VA_IDX();
        const int c4 = tid & 31;
        const bool act = tid < 32 && c4 < nc4;
        f32x4 lg = zv;
        if (act) {
#pragma unroll
          for (int gq = 0; gq < NG; ++gq) lg += red[gq * 32 + c4];
          lg += *reinterpret_cast<const f32x4*>(sb3 + 4 * c4);
        }
        int64_t lab;
        if constexpr (REM) {   // handed off by workgroup 0's receive: sc1 loads
          const __amdgpu_buffer_rsrc_t rY = rs_of(a.Yrem);
          const uint32_t lo = __builtin_bit_cast(uint32_t, hld1(rY, (i * M + m) * 8));
          const uint32_t hi = __builtin_bit_cast(uint32_t, hld1(rY, (i * M + m) * 8 + 4));
          lab = (int64_t)(((uint64_t)hi << 32) | lo);
        } else {
          lab = a.Y[(int64_t)i * M + m];
        }
        const bool ign = lab == a.ignore || lab < 0 || lab >= C;
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (act && 4 * c4 + c < C) mx = fmaxf(mx, lg[c]);
        mx = sl_wave_max(mx);
        f32x4 e = zv;
        float se = 0.f, zl = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int cc2 = 4 * c4 + c;
          if (act && cc2 < C) {
            e[c] = expf(lg[c] - mx);
            se += e[c];
            if (cc2 == lab) zl = lg[c];
          }
        }
        se = sl_wave_sum(se);
        zl = sl_wave_sum(zl);
        const float inv = 1.f / se;
        f32x4 d = zv;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int cc2 = 4 * c4 + c;
          float pr = e[c] * inv;
          if (cc2 == lab) pr -= 1.f;
          d[c] = (ign || cc2 >= C) ? 0.f : pr * a.adam[4 * i + 2];
        }
        if (act) hst4(rHB, bDL + ((par * 16 + m) * C4 + 4 * c4) * 4, d);
        if (tid == 0) a.loss[(int64_t)i * M + m] = ign ? 0.f : mx + logf(se) - zl;
      }
      va_arrive(a, va_seam(2, w & 7));
    }

    // ================= H2: dz2 of the head rows; b3 / W3 / b2 steps
    if (head) {
      if (!va_seam_wait(a, 2, (unsigned)(i + 1), s_ok, s_sn)) break;
      {
        VA_IDX();
        for (int e = tid; e < 16 * (MC / 4); e += kVaThreads) {
          const int m = e / (MC / 4), c = 4 * (e - m * (MC / 4));
          *reinterpret_cast<f32x4*>(sdl + m * MC + c) = (m < M && c < C4) ? hld4(rHB, bDL + ((par * 16 + m) * C4 + c) * 4) : zv;
        }
      }
      __syncthreads();
      {
        VA_IDX();
#pragma unroll
        for (int oi0 = 0; oi0 < 64; oi0 += kVaThreads / 16) {
          const int oi = oi0 + (tid >> 4), part = tid & 15;
          const int m = oi >> 2, ii = oi & 3;
          float s = 0.f;
#pragma unroll
          for (int c2 = 0; c2 < MC; c2 += 16) s = fmaf(sdl[m * MC + c2 + part], sW3[ii * MC + c2 + part], s);
          s = sl_row16_sum(s);
          if (part == 0) {
            const float h = sh2[m * 4 + ii];
            sdzh[m * 4 + ii] = (m < M && h > 0.f) ? s * a.dsc2 : 0.f;
          }
        }
      }
      __syncthreads();
      if (threadIdx.x < 16 && (int)threadIdx.x < M)
        hst4(rHB, bDZ + ((par * 16 + threadIdx.x) * N2 + 4 * w) * 4, *reinterpret_cast<const f32x4*>(sdzh + threadIdx.x * 4));
      va_arrive(a, va_seam(3, w & 7));
      {
        VA_IDX();
        float dummy = 0.f;
        if (tid < C) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdl[m * MC + tid];
          res_update<false>(o, ss, ib, sb3[tid], g, sb3[MC + tid], dummy);
        }
        for (int e = tid; e < 4 * MC; e += kVaThreads) {
          const int ii = e / MC, c = e - ii * MC;
          if (c < C) {
            float g = 0.f;
#pragma unroll
            for (int m = 0; m < 16; ++m) g = fmaf(sdl[m * MC + c], sh2[m * 4 + ii], g);
            res_update<false>(o, ss, ib, sW3[ii * MC + c], g, sW3[(4 + ii) * MC + c], dummy);
          }
        }
        if (tid < 4) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdzh[m * 4 + tid];
          res_update<false>(o, ss, ib, sb2[tid], g, sb2[4 + tid], dummy);
        }
      }
    }

    VA_MARK(3);
    // ================= B: the tile's dz1 partial, then W2's step
    if (!va_seam_wait(a, 3, (unsigned)(i + 1), s_ok, s_sn)) break;
    VA_MARK(3);
    {
      VA_IDX();
      const int m = tid >> 5, k4 = tid & 31;
      const f32x4 v = (m < M && 4 * k4 < WR) ? hld4(rHB, bDZ + ((par * 16 + m) * N2 + r0 + 4 * k4) * 4) : zv;
#pragma unroll
      for (int k = 0; k < 4; ++k) sdz2[m * PD + 4 * k4 + k] = v[k];
    }
    __syncthreads();
    {
      VA_IDX();
      const int jt0 = r, jt1 = r + 8;
      const bool two = 16 * jt1 < WC;
      if (16 * jt0 < WC) {
        f32x4 a0 = zv, a1 = zv, b0 = zv, b1 = zv;
        const float* pa = sdz2 + li * PD + lq;
        const float* pb0 = sw2 + lq * PW2 + 16 * jt0 + li;
        const float* pb1 = sw2 + lq * PW2 + 16 * (two ? jt1 : jt0) + li;
#pragma unroll
        for (int kk = 0; kk < kVaMaxWR / 4; kk += 2) {
          if (4 * kk < WR) {
            const float x = pa[4 * kk];
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb0[4 * kk * PW2], a0, 0, 0, 0);
            if (two) b0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb1[4 * kk * PW2], b0, 0, 0, 0);
          }
          if (4 * kk + 4 < WR) {
            const float x = pa[4 * kk + 4];
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb0[(4 * kk + 4) * PW2], a1, 0, 0, 0);
            if (two) b1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, pb1[(4 * kk + 4) * PW2], b1, 0, 0, 0);
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (h == 1 && !two) break;
          const f32x4 acc = h == 0 ? a0 + a1 : b0 + b1;
          const int j = 16 * (h == 0 ? jt0 : jt1) + li;
          if (j < WC) hst4(rHB, bDP + (((par * kVaNR + ta) * N1 + c0 + j) * 16 + 4 * lq) * 4, acc);
        }
      }
    }
    va_arrive(a, va_P(tb));
    VA_MARK(4);
    // the first update tile's state in flight under W2's update and the dz1 wait
    if (unt > 0) load_u(u_begin, sp[0], sm[0]);
    {
      VA_IDX();
      f32x4 dummy = zv;
#pragma unroll
      for (int u = 0; u < 10; ++u) {
        const int b = r + 8 * u, bn = b / 10, bk = b - (b / 10) * 10;
        if (16 * bn < WR && 16 * bk < WC) {
          f32x4 g = zv;
#pragma unroll
          for (int st = 0; st < 4; ++st)
            g = __builtin_amdgcn_mfma_f32_16x16x4f32(sdz2[(4 * st + lq) * PD + 16 * bn + li],
                                                     sh1[(4 * st + lq) * PH + 16 * bk + li], g, 0, 0, 0);
          f32x4 p;
#pragma unroll
          for (int j = 0; j < 4; ++j) p[j] = sw2[(16 * bn + 4 * lq + j) * PW2 + 16 * bk + li];
          res_update4<false>(o, ss, ib, p, g, m2[u], dummy);
#pragma unroll
          for (int j = 0; j < 4; ++j) sw2[(16 * bn + 4 * lq + j) * PW2 + 16 * bk + li] = p[j];
        }
      }
    }

    VA_MARK(5);
    // ================= U: dz1 of the update run and the forward run, b1's step, the update pass
    {
      // every fc2 column block's dz1 partials (the update run spans ~27 row blocks, possibly
      // wrapping to the next column block's top)
      if (!va_wait_many(a, NC, s_ok, [&](int l, int& idx) {
            idx = va_P(l);
            return (unsigned)(i + 1) * kVaNR;
          }))
        break;
    }
    VA_MARK(6);
    {
      VA_IDX();
      // (row nn, rows m = 4 mg ..): DP is [8][N1][16], H1 [N1][16]; up to 4 items per thread,
      // unrolled so that all their loads are in flight together (a rolled loop took 4.5 us)
#pragma unroll
      for (int u = 0; u < (kVaMaxRun + kVaRuns + 7) / 8; ++u) {
        const int e = tid + u * kVaThreads;
        const bool item = e < (unt + nruns) * 64;
        const int j = e >> 6, nn = (e >> 2) & 15, mg = e & 3;
        const bool upd = j < unt;
        const int rb = upd ? u_rb0 + (u_begin + j) - ((u_begin + j) / u_nb) * u_nb : rbA + (j - unt);
        const int n = 16 * rb + nn;
        f32x4 v = zv;
        if (item && n < N1) {
          f32x4 parts[kVaNR];
#pragma unroll
          for (int b = 0; b < kVaNR; ++b) parts[b] = hld4(rHB, bDP + (((par * kVaNR + b) * N1 + n) * 16 + 4 * mg) * 4);
          const f32x4 h = hld4(rHB, bH1 + ((par * N1 + n) * 16 + 4 * mg) * 4);
          v = parts[0];
#pragma unroll
          for (int b = 1; b < kVaNR; ++b) v += parts[b];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = (4 * mg + q < M && h[q] > 0.f) ? v[q] * a.dsc1 : 0.f;
        }
        float* dst = upd ? sdz1 + j * 256 : sdzb + (j - unt) * 256;
        if (item) {
#pragma unroll
          for (int q = 0; q < 4; ++q) dst[(4 * mg + q) * 16 + nn] = v[q];
        }
      }
    }
    __syncthreads();
    {
      VA_IDX();
      if (tid < 16 * nruns) {
        const int k = tid >> 4, jj = tid & 15;
        const int rb = rbA + k;
        if (s_slot[k] == 0 && 16 * rb + jj < N1) {
          float g = 0.f, dummy = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdzb[k * 256 + m * 16 + jj];
          res_update<false>(o, ss, ib, sb1[(k * 3) * 16 + jj], g, sb1[(k * 3 + 1) * 16 + jj], dummy);
        }
      }
    }
    __syncthreads();   // sdzb (union) is read before the update pass stages x over it
    VA_MARK(7);
    upd_pass(i, ss, ib);
    VA_MARK(8);

    if constexpr (REM) {
      // ================= C (remote Alice): dx_i to her, her activation of batch i + 1 in
      if (!send_dx(i)) break;
      VA_MARK(9);
      if (more) {
        if (!recv_act(i + 1)) break;
        va_arrive(a, va_seam(4, w & 7));
        VA_MARK(12);
        if constexpr (kVaFwdPre > 0) {
          if (!wait_all_xd(i)) break;
          fwd_prefetch();
        }
        if (!va_seam_wait(a, 4, (unsigned)(i + 2), s_ok, s_sn)) break;
        VA_MARK(13);
        ack_act(i + 1);
        fwd_pass(i + 1);
        VA_MARK(14);
        flush(i + 1);
        VA_MARK(15);
      }
      continue;
    }
    // ================= C: Alice's backward + step (conv job), her forward of batch i + 1
    {
      const int k0 = cc * 169, cblo = k0 >> 8, cbhi = (k0 + 168) >> 8;
      if (!va_wait_many(a, cbhi - cblo + 1, s_ok, [&](int l, int& idx) {
            idx = va_XD(cblo + l);
            return (unsigned)(i + 1) * (unsigned)a.tab[a.oU + cblo + l];
          }))
        break;
    }
    VA_MARK(9);
    img_put(par ^ 1, pimg);
    {
      VA_IDX();
      float acc[10];
#pragma unroll
      for (int j = 0; j < 10; ++j) acc[j] = 0.f;
      if (tid < 338) {
        const int bl = tid / 169, p = tid - (tid / 169) * 169;
        const int m = 2 * cg + bl;
        if (m < M && cy > 0.f) {
          const int k = cc * 169 + p, cb = k >> 8, kk = k & 255;
          const int ns = a.tab[a.oU + cb];
          float parts[kVaDxSlots];
#pragma unroll
          for (int s = 0; s < kVaDxSlots; ++s)
            parts[s] = s < ns ? hld1(rHB, bDX + (((cb * kVaDxSlots + s) * 16 + m) * 256 + kk) * 4) : 0.f;
          float gx = parts[0];
#pragma unroll
          for (int s = 1; s < kVaDxSlots; ++s) gx += parts[s];
          const uint8_t* im = simg + par * 1568 + bl * 784;
          const int ph = p / 13, pw = p - (p / 13) * 13;
          const int rr = 2 * ph + (carg >> 1), c2 = 2 * pw + (carg & 1);
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] = gx * (float)im[(rr + kh) * 28 + c2 + kw];
          acc[9] = gx;
        }
      }
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const float v = sl_wave_sum(acc[j]);
        if (lane == 0) scred[r * 16 + j] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x < 10) {
      const int j = threadIdx.x;
      float g = scred[j];
#pragma unroll
      for (int ww = 1; ww < 8; ++ww) g += scred[ww * 16 + j];
      hst1(rHB, bCW + (((par * 32 + cc) * 8 + cg) * 16 + j) * 4, g);
    }
    va_arrive(a, va_CW(cc));
    VA_MARK(10);
    if (!va_wait_many(a, 1, s_ok, [&](int, int& idx) {
          idx = va_CW(cc);
          return (unsigned)(i + 1) * 8u;
        }))
      break;
    VA_MARK(11);
    if (threadIdx.x < 10) {
      const int j = threadIdx.x;
      float parts[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) parts[q] = hld1(rHB, bCW + (((par * 32 + cc) * 8 + q) * 16 + j) * 4);
      float g = parts[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) g += parts[q];
      float p = scv[j], s0 = scv[10 + j], s1 = 0.f;
      sl_opt_update(a.oa, p, g, s0, s1);
      scv[j] = p;
      scv[10 + j] = s0;
    }
    __syncthreads();
    if (more) {
      conv_fwd(i + 1);
      if (!seam_x((unsigned)(i + 2), [&] {
            VA_MARK(12);
            if constexpr (kVaFwdPre > 0) {
              if (!wait_all_xd(i)) return false;
              fwd_prefetch();
            }
            return true;
          }))
        break;
      VA_MARK(13);
      // ================= V: the forward pass of batch i + 1 over the updated fc1
      fwd_pass(i + 1);
      VA_MARK(14);
      flush(i + 1);
      VA_MARK(15);
    }
  }

done:
  // ---- write the resident state back
  __syncthreads();
  {
    VA_IDX();
    for (int e = tid; e < WR * WC4; e += kVaThreads) {
      const int n = e / WC4, q = e - n * WC4;
      f32x4 wv;
#pragma unroll
      for (int k = 0; k < 4; ++k) wv[k] = sw2[n * PW2 + 4 * q + k];
      *reinterpret_cast<f32x4*>(a.L2.W + (int64_t)(r0 + n) * N1 + c0 + 4 * q) = wv;
    }
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int b = r + 8 * u, bn = b / 10, bk = b - (b / 10) * 10;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * bn + 4 * lq + j, k = 16 * bk + li;
        if (n < WR && k < WC) a.L2.m[(int64_t)(r0 + n) * N1 + c0 + k] = m2[u][j];
      }
    }
    if (head && tid < 4 * MC) {
      const int ii = tid / MC, c = tid - ii * MC;
      if (c < C) {
        const int64_t off = (int64_t)c * N2 + 4 * w + ii;
        a.L3.W[off] = sW3[ii * MC + c];
        a.L3.m[off] = sW3[(4 + ii) * MC + c];
      }
    }
    if (w == 0 && tid < C) {
      a.L3.b[tid] = sb3[tid];
      a.L3.mb[tid] = sb3[MC + tid];
    }
    if (head && tid < 4) {
      const int n = 4 * w + tid;
      a.L2.b[n] = sb2[tid];
      a.L2.mb[n] = sb2[4 + tid];
    }
    if (tid < 16 * nruns) {
      const int k = tid >> 4, j = tid & 15;
      const int rb = rbA + k, n = 16 * rb + j;
      if (a.tab[G + 1 + rb] == w && n < N1) {
        a.L1.b[n] = sb1[(k * 3 + 0) * 16 + j];
        a.L1.mb[n] = sb1[(k * 3 + 1) * 16 + j];
      }
    }
    if (!REM && cg == 0 && tid < 20) {
      const int j = tid < 10 ? tid : tid - 10;
      float* dst = tid < 10 ? (j < 9 ? a.cw + cc * 9 + j : a.cb + cc) : (j < 9 ? a.cmw + cc * 9 + j : a.cmb + cc);
      *dst = scv[tid];
    }
  }
}
#undef VA_IDX
#undef VA_MARK

int vanilla_lds_bytes() { return kVaLds; }

std::string vanilla_check(const VaArgs& a) {
  if (a.M < 1 || a.M > 16) return "rows per step 1..16";
  if (a.rem) {
    if (a.G < kVaNR || a.G > kVaG || a.G % kVaNR || a.NC != a.G / kVaNR) return "remote Alice: 8..256 workgroups, a multiple of 8";
    if (a.M > a.G) return "remote Alice: a softmax workgroup per row";
    if (a.Yrem == nullptr || a.lk.sdata[0] == nullptr || a.lk.rdata[0] == nullptr) return "remote Alice: the channel";
  } else if (a.G != kVaG || a.NC != a.G / kVaNR || a.NC > kVaMaxNC) {
    return "256 workgroups (32 conv channels x 8 image pairs)";
  }
  if (a.N1 < 4 || a.N1 % 4) return "fc1 width % 4";
  if ((a.N1 / 4 + a.NC - 1) / a.NC > kVaMaxWC4) return "fc1 too wide for the fc2 tiles";
  if (a.N1 > 16 * kVaMaxRB || a.nrb != (a.N1 + 15) / 16) return "fc1 row blocks";
  if (a.K1 != 5408 || a.ncb != (a.K1 + 255) / 256 || a.ncb > kVaMaxCB) return "fc1 input width 5408 (32 x 13 x 13)";
  if ((int64_t)a.N1 * a.K1 * 4 > 2147483647LL) return "fc1 larger than 2 GB (32-bit buffer offsets)";
  if (a.N2 < 4 || a.N2 % 4 || a.N2 > 4 * a.G || 4 * ((a.N2 / 4 + kVaNR - 1) / kVaNR) > kVaMaxWR || a.HW != a.N2 / 4)
    return "fc2 width % 4, <= 1024";
  if (a.C < 1 || a.C > kVaMaxC || a.C4 != ((a.C + 3) & ~3)) return "classes <= 128";
  if (a.o.kind != 1 || a.oa.kind != 1) return "SGD-momentum on both sides";
  if (a.S > kVaMaxS) return "more than 6000 steps in one launch";
  return "";
}

bool vanilla_fits(const VaArgs& a, int device, std::string* why) {
  std::string s = vanilla_check(a);
  if (s.empty()) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, device) != hipSuccess) {
      s = "device properties";
    } else {
      const void* fn = a.rem ? reinterpret_cast<const void*>(&vanilla_epoch_kernel<true>)
                             : reinterpret_cast<const void*>(&vanilla_epoch_kernel<false>);
      int nb = 0;
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kVaLds);
      if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kVaThreads, kVaLds);
      if (e != hipSuccess || nb < 1) s = "occupancy";
      else if ((int64_t)nb * pr.multiProcessorCount < a.G) s = "workgroups not co-resident";
    }
  }
  if (why) *why = s;
  return s.empty();
}

hipError_t vanilla_epoch_launch(const VaArgs& a, hipStream_t st) {
  if (!vanilla_check(a).empty()) return hipErrorInvalidValue;
  if (a.S <= 0) return hipSuccess;
  const void* fn = a.rem ? reinterpret_cast<const void*>(&vanilla_epoch_kernel<true>)
                         : reinterpret_cast<const void*>(&vanilla_epoch_kernel<false>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kVaLds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.cnt, 0, (size_t)kVaCounters * kVaStride * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  VaArgs arg = a;
  void* params[] = {&arg};
  if (!a.coop) return hipLaunchKernel(fn, dim3(a.G), dim3(kVaThreads), params, (size_t)kVaLds, st);
  return hipLaunchCooperativeKernel(fn, dim3(a.G), dim3(kVaThreads), params, (unsigned)kVaLds, st);
}

}  // namespace sl
