// U-shape persistent split epoch: every batch of a co-located Alice's U-shape epoch in ONE
// launch, with every parameter and Adam moment on-chip for the whole epoch.
//
// Reference: the U-shape hot loop (data_entities.py:65-81): per batch, Alice's model1 forward
// (Conv2d(1, 32, 3) -> ReLU -> MaxPool(2, 2), models.py:5-14), Bob's model2 (fc1 5408 -> 1000
// ReLU, fc2 1000 -> 100 ReLU, models.py:33-44), Alice's model3 (fc3 100 -> 10, models.py:87-94)
// and the CE on Alice, the distributed backward through all three, and one Adam step of every
// parameter (data_entities.py:43-47: DistributedOptimizer(Adam) over model3 + model2 + model1).
//
// Why.  The launch-per-stage U-shape batch is ~10 dependent launches, 72 us on an MI355X, of
// which the fc1 wgrad + Adam stream (W / m / v of 5.4 M parameters, 130 MB per step) is the
// largest; the host issues the batch in ~60 us (profiles/r5w_misc/split_host_issue_probe.txt).
// 256 CUs hold 128 MiB of VGPRs: fc1's W / m / v (65 MB) fit in half of them.  Here workgroup
// w = (row group rg = w >> 5, channel c = w & 31) holds fc1 rows [128 rg, 128 rg + 128) x the 169
// columns of conv channel c (padded to 176) in registers for the whole epoch, so no fc1 byte
// moves between steps; a step moves only activations, partial sums and gradients.
//
// Ownership (thread: wave r, lane (li, lq) = (lane % 16, lane / 16)):
//   fc1   W / m / v [n = 128 rg + 16 r + li][169 c + 16 kb + 4 lq + comp] as Wr / Mr / Vr[kb][comp]
//         (kb < 11): the forward product's MFMA B operand as held, and exactly the lane layout of
//         the weight-gradient MFMA's output, so neither needs a register shuffle;
//   fc2   W2[:, n] for the workgroup's 4 fc1 rows n = 128 rg + 4 c + q (LDS, with m / v), b1[n];
//         b2[j] on workgroup j < N2;
//   head  W3 / b3 (model3) replicated on every workgroup (every copy takes the same step);
//   conv  channel c's 9 weights + bias (replicated on the channel's 8 workgroups); workgroup
//         (rg, c) is the conv job for images 2 rg, 2 rg + 1 of channel c.
// Step i (every hand-off: write-through (sc1) stores, drained, one agent-scope counter add per
// workgroup; consumers poll, barrier, sc1 loads -- MI355X_MICROARCH.md's valid-forms row 1,
// stress-tested by csrc/handoff.hip):
//   F   x_i of channel c (its 8 conv jobs' output) -> LDS; P[m][n] over the channel's columns
//       (exact-fp32 MFMA from the registers) -> PP; arrival on PC[rg]
//   R   the row group's 32 channel partials of my 4 rows -> h1 = relu(. + b1); the fc2 partial
//       over them P2[m][j] -> P2; arrival on the F2 shards
//   H2  workgroup j < N2: h2[:, j] = relu(sum of the 256 partials + b2[j]) -> H2; L shards
//   CE  workgroup m < M: logits of row m (model3), softmax-CE, dlogits -> DL, the row's loss
//   D   every workgroup: dz2 = dlog W3 masked by h2 > 0 (old W3), dz1 of my 4 rows = dz2 W2
//       masked by h1 > 0 (old W2) -> DZ; arrival on DZ[rg]; then (off the critical path) the
//       Adam steps of my W2 columns, b1, b2, and the replicated head
//   X   the row group's dz1 slab -> LDS, old W1 staged in LDS, the cut-gradient partial over my
//       128 rows dx[m][k] (exact-fp32 MFMA) -> DX; arrival on DX[c]
//   C   conv job: dx of its 2 images x 169 positions (the 8 row groups' partials in order), the
//       pool / ReLU backward (argmax kept in VGPRs since the forward), 10 conv gradients -> CW,
//       then the channel's 8 partials in order, the conv Adam step (every copy identically), the
//       conv forward of batch i + 1 -> XS; arrival on XC[c]
//   U   fc1's Adam step in registers: dW = dz1^T x_i on exact-fp32 MFMA, straight into the
//       lane's (row, column) layout
// Every sum runs in a fixed order: a launch is deterministic and one launch of S steps is
// bitwise S one-step launches.  Results agree with the per-batch executor and torch to fp32
// rounding (different summation orders; the hardware square root / reciprocal in Adam).
//
// REMOTE Alice (the <.., true> instantiations; BASELINE config 2: one Bob and one Alice on two
// GPUs, reference data_entities.py:65-81 over RPC).  Her conv front and head run in her process
// (csrc/split.cpp run_alice, unchanged) and the launch exchanges run_bob's four messages per step
// on the peer-mapped channel (csrc/ipc_p2p.h) itself, in place of the conv jobs and the CE:
//   in   her activation of step i: workgroup (rg, c) copies rows rg + RG t of channel c's slice
//        into XS (flags polled relaxed, one acquire, system-scope loads) -> XC[c];
//   out  h2 after the L shards (workgroups 0, 1: its <= 2 chunks, gathered from H2);
//   in   her premasked dz2 (every workgroup reads the <= 2 chunks into its dz2 slab) -> D;
//   out  the cut gradient after every channel's DX partials (workgroup c: chunk c, the row
//        groups' partials summed in order, as the conv jobs sum them).
// Sends are system-scope write-through stores, drained, released, then the chunk's flag; each
// send first waits for her ack of the message two generations back.  Her activation and dz2 of
// step i - 1 are acked at step i after the F2 seam (every workgroup has read them by then), the
// last dz2 after a closing seam.  Without conv jobs the grid is 32 RG workgroups for RG row groups
// (a one-GPU test runs a narrower fc1 on 64 CUs next to her kernels).
#include "ushape.h"
#include "ipc_ar.h"
#include "persist.h"

#include <string>

namespace sl {

namespace {

using namespace persist;

__device__ __forceinline__ unsigned* us_cnt(const UsArgs& a, int i) { return a.cnt + i * kUsStride; }

__device__ __forceinline__ bool us_spin(const UsArgs& a, const unsigned* p, unsigned tgt) {
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

// every wave drains its write-through stores, the barrier orders the drains before lane 0's add
__device__ __forceinline__ void us_arrive(const UsArgs& a, int idx) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(us_cnt(a, idx), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0's lanes [0, n) wait for counters tgt_of(lane, idx); the barrier then releases every
// wave to its sc1 loads.  Uniform result (false: a wait gave up)
template <typename F>
__device__ __forceinline__ bool us_wait(const UsArgs& a, int n, int* s_ok, F tgt_of) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < n) {
      int idx;
      const unsigned tg = tgt_of(lane, idx);
      if (tg > 0) ok = us_spin(a, us_cnt(a, idx), tg);
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  asm volatile("" ::: "memory");
  return *s_ok != 0;
}

// one lane: bounded wait until the channel flag / ack word *f reaches generation `want` (remote
// Alice); a timeout raises the launch's error word and the channel's
__device__ __forceinline__ bool us_pwait(const UsArgs& a, const uint32_t* f, uint32_t want) {
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

// arrivals per shard s of a seam whose producers are workgroups 0 .. n - 1 (shard w % 8)
__device__ __forceinline__ unsigned us_shard_n(int n, int s) { return n > s ? (unsigned)((n - 1 - s) / 8 + 1) : 0u; }

// LDS carve (bytes)
constexpr int US_SX = 0;                                  // x_i [16 m][176] (the step's channel slice)
constexpr int US_DZ1 = US_SX + 16 * kUsKP * 4;            // dz1 slab [16 m][132] (rows of the row group)
constexpr int kDzP = 132;
constexpr int US_U = US_DZ1 + 16 * kDzP * 4;              // union:
constexpr int U_WS = 0;                                   //   fc1 view: old W1 [128][176]
constexpr int kUWs = 128 * kUsKP * 4;
constexpr int U_SH2 = 0;                                  //   head view: h2 [16][128], dz2 [16][128],
constexpr int U_SDZ2 = U_SH2 + 16 * kUsN2P * 4;           //   reduction scratch [512 + 64] f32x4
constexpr int U_RED = U_SDZ2 + 16 * kUsN2P * 4;
constexpr int kUHead = U_RED + (512 + 64) * 16;
constexpr int kUU = kUWs > kUHead ? kUWs : kUHead;
constexpr int US_W2 = US_U + kUU;                         // W2[:, my 4 rows] {W, m, v}[4 q][128 j]
constexpr int US_W3 = US_W2 + 3 * 4 * kUsN2P * 4;         // W3 {W, m, v}[kUsW3]
constexpr int US_B3 = US_W3 + 3 * kUsW3 * 4;              // b3 {W, m, v}[16]
constexpr int US_B2 = US_B3 + 3 * kUsCP * 4;              // b2[j = w] {W, m, v, -}
constexpr int US_B1 = US_B2 + 16;                         // b1 of my 4 rows {W, m, v}[4]
constexpr int US_H1 = US_B1 + 3 * 4 * 4;                  // h1 of my 4 rows [16 m][4]
constexpr int US_DZM = US_H1 + 16 * 4 * 4;                // dz1 of my 4 rows [16 m][4]
constexpr int US_DL = US_DZM + 16 * 4 * 4;                // dlogits [16 m][16]
constexpr int US_LG = US_DL + 16 * kUsCP * 4;             // logits of the CE row [16]
constexpr int US_IMG = US_LG + kUsCP * 4;                 // images [2 parity][2][784] bytes
constexpr int US_CV = US_IMG + 2 * 2 * 784;               // conv channel {w9, b, m10, v10} (+ pad)
constexpr int US_CRED = US_CV + 32 * 4;                   // conv gradient reduction [8 waves][16]
constexpr int US_OK = US_CRED + 8 * 16 * 4;
constexpr int kUsLds = US_OK + 16;
static_assert(kUsLds <= 160 * 1024, "LDS");
static_assert(US_IMG % 16 == 0 && US_CV % 16 == 0 && US_W3 % 16 == 0 && US_DL % 16 == 0, "alignment");

}  // namespace

#define US_IDX()                                                           \
  int tid_l_ = threadIdx.x;                                                \
  asm volatile("" : "+v"(tid_l_));                                         \
  const int tid = tid_l_, r = tid >> 6, lane = tid & 63, li = lane & 15, lq = lane >> 4; \
  (void)r; (void)lane; (void)li; (void)lq

// BF (`--dtype bf16`): every product's operands rounded to bf16 with fp32 accumulation, as the
// per-batch executor's bf16 kernels (linear.hip / fused.hip / loss.hip); fc1's three products on
// bf16 MFMA (v_mfma_f32_16x16x16_bf16: one instruction per 16-column block where the fp32 form
// issues four), the conv front in fp32 (as conv.hip), every state and moment fp32.
typedef __bf16 us_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ us_bf16x4 us_bf4(f32x4 v) {
  return us_bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}

// REM: the Alice is remote (the channel phases above in place of her conv jobs and head)
template <bool BF, bool REM>
__global__ void __launch_bounds__(kUsThreads) ushape_epoch_kernel(UsArgs a) {
  auto R = [](float v) { return BF ? bfr(v) : v; };
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sx = reinterpret_cast<float*>(smem + US_SX);
  float* sdz = reinterpret_cast<float*>(smem + US_DZ1);
  float* sws = reinterpret_cast<float*>(smem + US_U + U_WS);
  float* sh2 = reinterpret_cast<float*>(smem + US_U + U_SH2);
  float* sdz2 = reinterpret_cast<float*>(smem + US_U + U_SDZ2);
  f32x4* red = reinterpret_cast<f32x4*>(smem + US_U + U_RED);
  float* sW2 = reinterpret_cast<float*>(smem + US_W2);
  float* sW3 = reinterpret_cast<float*>(smem + US_W3);
  float* sb3 = reinterpret_cast<float*>(smem + US_B3);
  float* sb2 = reinterpret_cast<float*>(smem + US_B2);
  float* sb1 = reinterpret_cast<float*>(smem + US_B1);
  float* sh1 = reinterpret_cast<float*>(smem + US_H1);
  float* sdzm = reinterpret_cast<float*>(smem + US_DZM);
  float* sdl = reinterpret_cast<float*>(smem + US_DL);
  float* slg = reinterpret_cast<float*>(smem + US_LG);
  uint8_t* simg = reinterpret_cast<uint8_t*>(smem + US_IMG);
  float* scv = reinterpret_cast<float*>(smem + US_CV);
  float* scred = reinterpret_cast<float*>(smem + US_CRED);
  int* s_ok = reinterpret_cast<int*>(smem + US_OK);
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};

  const int w = blockIdx.x, rg = w >> 5, cc = w & 31;
  const int M = a.M, N1 = a.N1, N2 = a.N2, C = a.C;
  const int RG = REM ? a.RG : kUsRG, G = REM ? a.G : kUsG;
  const int nb = 128 * rg;
  const __amdgpu_buffer_rsrc_t rHB = rs_of(a.HB);
  const int bXS = 4 * a.oXS, bPP = 4 * a.oPP, bP2 = 4 * a.oP2, bH2 = 4 * a.oH2, bDL = 4 * a.oDL, bDZ = 4 * a.oDZ,
            bDX = 4 * a.oDX, bCW = 4 * a.oCW;

  // ---- the state: fc1 block in registers, the rest in LDS
  f32x4 Wr[kUsKB], Mr[kUsKB], Vr[kUsKB];
  {
    US_IDX();
    const int n = nb + 16 * r + li;
#pragma unroll
    for (int kb = 0; kb < kUsKB; ++kb)
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) {
        const int lc = 16 * kb + 4 * lq + comp;
        const bool ok = n < N1 && lc < kUsP;
        const int64_t off = (int64_t)n * (kUsCh * kUsP) + kUsP * cc + lc;
        Wr[kb][comp] = ok ? a.W1[off] : 0.f;
        Mr[kb][comp] = ok ? a.m1[off] : 0.f;
        Vr[kb][comp] = ok ? a.v1[off] : 0.f;
      }
    {
      const int q = tid >> 7, j = tid & 127, n2 = nb + 4 * cc + q;
      const bool ok = n2 < N1 && j < N2;
      const int64_t off = (int64_t)j * N1 + n2;
      sW2[q * 128 + j] = ok ? a.W2[off] : 0.f;
      sW2[512 + q * 128 + j] = ok ? a.m2[off] : 0.f;
      sW2[1024 + q * 128 + j] = ok ? a.v2[off] : 0.f;
    }
    for (int e = tid; !REM && e < kUsW3; e += kUsThreads) {
      const bool ok = e < C * N2;
      sW3[e] = ok ? a.W3[e] : 0.f;
      sW3[kUsW3 + e] = ok ? a.m3[e] : 0.f;
      sW3[2 * kUsW3 + e] = ok ? a.v3[e] : 0.f;
    }
    if (!REM && tid < kUsCP) {
      const bool ok = tid < C;
      sb3[tid] = ok ? a.b3[tid] : 0.f;
      sb3[kUsCP + tid] = ok ? a.mb3[tid] : 0.f;
      sb3[2 * kUsCP + tid] = ok ? a.vb3[tid] : 0.f;
    }
    if (tid < 4) {
      const int n1 = nb + 4 * cc + tid;
      const bool ok = n1 < N1;
      sb1[tid] = ok ? a.b1[n1] : 0.f;
      sb1[4 + tid] = ok ? a.mb1[n1] : 0.f;
      sb1[8 + tid] = ok ? a.vb1[n1] : 0.f;
    }
    if (tid == 0) {
      const bool ok = w < N2;
      sb2[0] = ok ? a.b2[w] : 0.f;
      sb2[1] = ok ? a.mb2[w] : 0.f;
      sb2[2] = ok ? a.vb2[w] : 0.f;
    }
    if (!REM && tid < 10) {
      // {w[9], b} of channel cc, then their m, then their v
      const int j = tid;
      scv[j] = j < 9 ? a.cw[cc * 9 + j] : a.cb[cc];
      scv[10 + j] = j < 9 ? a.cmw[cc * 9 + j] : a.cmb[cc];
      scv[20 + j] = j < 9 ? a.cvw[cc * 9 + j] : a.cvb[cc];
    }
  }

  // ---- the conv job: channel cc of images 2 rg, 2 rg + 1
  auto img_word = [&](int step) -> uint32_t {
    US_IDX();
    uint32_t v = 0;
    if (tid < 392 && step < a.S) {
      const int bl = tid / 196, wd = tid - (tid / 196) * 196;
      const int m = 2 * rg + bl;
      const int64_t src = m < M ? a.rows[(int64_t)step * M + m] : -1;
      if (src >= 0) v = reinterpret_cast<const uint32_t*>(a.img + src * 784)[wd];
    }
    return v;
  };
  auto img_put = [&](int par, uint32_t v) {
    US_IDX();
    if (tid < 392) reinterpret_cast<uint32_t*>(simg + par * 1568)[tid] = v;
  };
  // pooled output (image bl, position p) of channel cc over image buffer par (conv.hip's
  // arithmetic: the first maximum in torch's window order, then ReLU)
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
  float cy = 0.f;
  int carg = 0;
  auto conv_fwd = [&](int step) {
    US_IDX();
    if (tid < 2 * kUsP) {
      const int bl = tid / kUsP, p = tid - (tid / kUsP) * kUsP;
      const int m = 2 * rg + bl;
      const bool valid = m < M && a.rows[(int64_t)step * M + m] >= 0;
      float y = 0.f;
      int arg = 0;
      if (valid) conv_at(step & 1, bl, p, y, arg);
      cy = y;
      carg = arg;
      if (m < M) hst1(rHB, bXS + ((((step & 1) * kUsCh + cc) * 16 + m) * kUsKP + p) * 4, y);
    }
  };

  // ---------------------------------------------------------------- remote Alice (REM)
  auto rows_of = [&](int s) { return (int)a.tabf[8 * s + 5]; };
  auto nchunks = [](int n) { return (n + kIpcChunk - 1) / kIpcChunk; };
  // her activation of step s -> XS[s & 1]: workgroup (rg, cc) rows m = rg + RG t (t < 16 / RG) of
  // channel cc's 169 columns (padding rows zero); false when a wait gave up
  auto recv_act = [&](int s) -> bool {
    const int Ms = rows_of(s);
    const uint32_t gen = a.lk.rgen0 + 1u + 2u * (uint32_t)s;
    const int par = (int)(gen & 1u);
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x, t = lane >> 1, m = rg + RG * t;
      bool ok = true;
      if (t < 16 / RG && m < Ms) {
        const int base = m * (kUsCh * kUsP) + cc * kUsP;
        ok = us_pwait(a, a.lk.rflag[par] + ((lane & 1) ? base + kUsP - 1 : base) / kIpcChunk, gen);
      }
      ok = __all(ok);
      ipc_acquire();
      if (lane == 0) *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (*s_ok == 0) return false;
    const __amdgpu_buffer_rsrc_t rR = ipc_rsrc(a.lk.rdata[par]);
    for (int e = threadIdx.x; e < (16 / RG) * kUsP; e += kUsThreads) {
      const int t = e / kUsP, p = e - t * kUsP, m = rg + RG * t;
      float v = 0.f;
      if (m < Ms)
        v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rR, (m * (kUsCh * kUsP) + cc * kUsP + p) * 4, 0, 17));
      hst1(rHB, bXS + ((((s & 1) * kUsCh + cc) * 16 + m) * kUsKP + p) * 4, v);
    }
    return true;
  };
  // one chunk of a message to her: wait for her ack of the message two generations back on the
  // slot, fill(e, v) -> the float4 at e (< len), system-scope stores, drain, release, flag
  auto send_chunk = [&](int c, uint32_t gen, int prev, int len, auto fill) -> bool {
    const int par = (int)(gen & 1u);
    if (threadIdx.x == 0) {
      const bool ok = prev == 0 || us_pwait(a, a.lk.sack[par] + (c < prev ? c : 0), gen - 2u);
      ipc_acquire();
      *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (*s_ok == 0) return false;
    const int e = c * kIpcChunk + 4 * (int)threadIdx.x;
    if ((int)threadIdx.x < kIpcThreads && e < len) ipc_st4(ipc_rsrc(a.lk.sdata[par]), e, __builtin_bit_cast(float4, fill(e)));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) ipc_raise_flag(a.lk.sflag[par] + c, gen);
    __syncthreads();
    return true;
  };
  int i_end = 0;   // steps completed (remote: the closing ack)

  // ---- prologue: Alice's forward of batch 0 (remote: her message of it)
  if constexpr (REM) {
    if (!recv_act(0)) goto fin;
  } else {
    img_put(0, img_word(0));
    __syncthreads();
    conv_fwd(0);
  }
  us_arrive(a, kUsXC + cc);

  for (int i = 0; i < a.S; ++i) {
    const int par = i & 1;
    const bool more = i + 1 < a.S;
    float ss_b = a.tabf[8 * i], ib_b = a.tabf[8 * i + 1], ss_a = a.tabf[8 * i + 2], ib_a = a.tabf[8 * i + 3];
    const float cs = a.tabf[8 * i + 4];
    asm volatile("" : "+v"(ss_b), "+v"(ib_b), "+v"(ss_a), "+v"(ib_a));   // held in VGPRs (res_update)
    // the next batch's images, in flight across the step (into LDS in the conv phase)
    const uint32_t pimg = (!REM && more) ? img_word(i + 1) : 0u;

    // ================= F: x_i of channel cc, the forward partial over its columns
    if (!us_wait(a, 1, s_ok, [&](int, int& idx) {
          idx = kUsXC + cc;
          return i == a.fault_step ? 0xffffffffu : (unsigned)RG * (unsigned)(i + 1);
        }))
      break;
    {
      US_IDX();
      for (int e = tid; e < 16 * (kUsKP / 4); e += kUsThreads) {
        const int m = e / (kUsKP / 4), q = e - m * (kUsKP / 4);
        *reinterpret_cast<f32x4*>(sx + m * kUsKP + 4 * q) =
            hld4(rHB, bXS + (((par * kUsCh + cc) * 16 + m) * kUsKP + 4 * q) * 4);
      }
    }
    __syncthreads();
    {
      // P[m][n = 16 r + li] over columns 16 kb + 4 lq + comp (MFMA comp: A = x[li][..], B = Wr)
      US_IDX();
      f32x4 acc0 = zv, acc1 = zv;
#pragma unroll
      for (int kb = 0; kb < kUsKB; ++kb) {
        const f32x4 xa = *reinterpret_cast<const f32x4*>(sx + li * kUsKP + 16 * kb + 4 * lq);
        if constexpr (BF) {
          // k = 4 lq + comp of the block: the fp32 form's four instructions as one
          if (kb & 1)
            acc1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(us_bf4(xa), us_bf4(Wr[kb]), acc1, 0, 0, 0);
          else
            acc0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(us_bf4(xa), us_bf4(Wr[kb]), acc0, 0, 0, 0);
          asm volatile("" ::: "memory");
          continue;
        }
#pragma unroll
        for (int comp = 0; comp < 4; ++comp) {
          if (kb & 1)
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[comp], Wr[kb][comp], acc1, 0, 0, 0);
          else
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[comp], Wr[kb][comp], acc0, 0, 0, 0);
        }
        asm volatile("" ::: "memory");   // one k-block's operands live at a time (VGPR budget)
      }
      acc0 += acc1;   // lane: P[m = 4 lq + j][n = 16 r + li]
      hst4(rHB, bPP + ((((par * kUsRG + rg) * kUsCh + cc) * 128 + 16 * r + li) * 16 + 4 * lq) * 4, acc0);
    }
    us_arrive(a, kUsPC + rg);

    // ================= R: h1 of my 4 rows, the fc2 partial over them
    if (!us_wait(a, 1, s_ok, [&](int, int& idx) {
          idx = kUsPC + rg;
          return 32u * (unsigned)(i + 1);
        }))
      break;
    {
      US_IDX();
      const int cp = tid >> 4, o = tid & 15, q = o >> 2, mg = o & 3;
      red[tid] = hld4(rHB, bPP + ((((par * kUsRG + rg) * kUsCh + cp) * 128 + 4 * cc + q) * 16 + 4 * mg) * 4);
    }
    __syncthreads();
    {
      US_IDX();
      if (tid < 16) {
        const int q = tid >> 2, mg = tid & 3;
        f32x4 s = red[tid];
        // (not unrolled: 31 hoisted f32x4 loads would not fit the VGPRs the fc1 block leaves)
#pragma unroll 1
        for (int cp = 1; cp < kUsCh; ++cp) s += red[cp * 16 + tid];
        const bool ok = nb + 4 * cc + q < N1;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) sh1[(4 * mg + jj) * 4 + q] = ok ? fmaxf(s[jj] + sb1[q], 0.f) : 0.f;
      }
    }
    __syncthreads();
    {
      US_IDX();
      const int j = tid >> 2, mg = tid & 3;
      f32x4 p = zv;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float w2 = R(sW2[q * 128 + j]);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) p[jj] = fmaf(R(sh1[(4 * mg + jj) * 4 + q]), w2, p[jj]);
      }
      hst4(rHB, bP2 + (((par * kUsN2P + j) * kUsG + w) * 16 + 4 * mg) * 4, p);
    }
    us_arrive(a, kUsF2 + (w & 7));

    // ================= H2: workgroup j = w < N2 reduces fc2 column j
    if (w < N2) {
      if (!us_wait(a, 8, s_ok, [&](int l, int& idx) {
            idx = kUsF2 + l;
            return (unsigned)(G / 8) * (unsigned)(i + 1);
          }))
        break;
      if constexpr (REM) {
        // every workgroup has read her activation of this step and her dz2 of the last one
        if (threadIdx.x == 0) {
          const uint32_t ga = a.lk.rgen0 + 1u + 2u * (uint32_t)i;
          for (int c = w; c < nchunks(rows_of(i) * (kUsCh * kUsP)); c += N2)
            ipc_raise_flag(a.lk.rack[ga & 1u] + c, ga, 0);
          if (i > 0) {
            const uint32_t gd = ga - 1u;
            for (int c = w; c < nchunks(rows_of(i - 1) * N2); c += N2) ipc_raise_flag(a.lk.rack[gd & 1u] + c, gd, 0);
          }
        }
      }
      {
        US_IDX();
        const int sl = tid >> 2, mg = tid & 3;   // producers 2 sl, 2 sl + 1
        const f32x4 u0 = hld4(rHB, bP2 + (((par * kUsN2P + w) * kUsG + 2 * sl) * 16 + 4 * mg) * 4);
        const f32x4 u1 = hld4(rHB, bP2 + (((par * kUsN2P + w) * kUsG + 2 * sl + 1) * 16 + 4 * mg) * 4);
        red[tid] = u0 + u1;
      }
      __syncthreads();
      {
        US_IDX();
        if (tid < 64) {
          const int mg = tid & 3, gp = tid >> 2;
          f32x4 s = red[(gp * 8) * 4 + mg];
#pragma unroll
          for (int k = 1; k < 8; ++k) s += red[(gp * 8 + k) * 4 + mg];
          red[512 + tid] = s;
        }
      }
      __syncthreads();
      {
        US_IDX();
        if (tid < 4) {
          f32x4 s = red[512 + tid];
#pragma unroll
          for (int gp = 1; gp < 16; ++gp) s += red[512 + gp * 4 + tid];
          f32x4 h;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) h[jj] = fmaxf(s[jj] + sb2[0], 0.f);
          hst4(rHB, bH2 + ((par * kUsN2P + w) * 16 + 4 * tid) * 4, h);
        }
      }
      us_arrive(a, kUsL + (w & 7));
    }

    // ================= (remote) h2 to her: workgroups c < its chunks, after the L shards
    if constexpr (REM) {
      const int len = rows_of(i) * N2;
      if (w < nchunks(len)) {
        if (!us_wait(a, 8, s_ok, [&](int l, int& idx) {
              idx = kUsL + l;
              return (unsigned)(i + 1) * us_shard_n(N2, l);
            }))
          break;
        const uint32_t gen = a.lk.sgen0 + 1u + 2u * (uint32_t)i;
        const int prev = i > 0 ? nchunks(rows_of(i - 1) * N2) : a.lk.sprev[0];
        if (!send_chunk(w, gen, prev, len, [&](int e) {
              const int m = e / N2, j = e - m * N2;   // N2 % 4 == 0: one row
              f32x4 v;
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = hld1(rHB, bH2 + ((par * kUsN2P + j + q) * 16 + m) * 4);
              return v;
            }))
          break;
      }
    }
    // ================= CE: workgroup m = w < M: model3 logits of row m, softmax-CE, dlogits
    if (!REM && w < M) {
      if (!us_wait(a, 8, s_ok, [&](int l, int& idx) {
            idx = kUsL + l;
            return (unsigned)(i + 1) * us_shard_n(N2, l);
          }))
        break;
      {
        US_IDX();
        if (tid < kUsN2P) sh2[tid] = tid < N2 ? hld1(rHB, bH2 + ((par * kUsN2P + tid) * 16 + w) * 4) : 0.f;
      }
      __syncthreads();
      {
        US_IDX();
        if (tid < 16 * kUsCP) {
          const int cls = tid >> 4, part = tid & 15;
          float s = 0.f;
          if (cls < C)
            for (int j = part; j < N2; j += 16) s = fmaf(R(sh2[j]), R(sW3[cls * N2 + j]), s);
          s = sl_row16_sum(s);
          if (part == 0) slg[cls] = s + sb3[cls];
        }
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        const int cls = threadIdx.x;
        const bool act = cls < C;
        const float lg = act ? slg[cls] : 0.f;
        const int64_t lab = a.Y[(int64_t)i * M + w];
        const bool ign = lab == a.ignore || lab < 0 || lab >= C;
        const float mx = sl_wave_max(act ? lg : -INFINITY);
        const float e = act ? expf(lg - mx) : 0.f;
        const float se = sl_wave_sum(e);
        const float zl = sl_wave_sum(act && cls == lab ? lg : 0.f);
        float pr = e * (1.f / se);
        if (cls == lab) pr -= 1.f;
        if (cls < kUsCP) hst1(rHB, bDL + ((par * 16 + w) * kUsCP + cls) * 4, (ign || !act) ? 0.f : pr * cs);
        if (cls == 0) a.loss[(int64_t)i * M + w] = ign ? 0.f : mx + logf(se) - zl;
      }
      us_arrive(a, kUsD + (w & 7));
    }

    // ================= D: dz2 (old head), dz1 of my 4 rows (old W2); then the small Adam steps
    if constexpr (REM) {
      // her premasked dz2 (scaled by her CE) -> the dz2 slab
      const int Mi = rows_of(i), len = Mi * N2;
      const uint32_t gen = a.lk.rgen0 + 2u + 2u * (uint32_t)i;
      if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const bool ok = __all(lane < nchunks(len) ? us_pwait(a, a.lk.rflag[gen & 1u] + lane, gen) : true);
        ipc_acquire();
        if (lane == 0) *s_ok = ok ? 1 : 0;
      }
      __syncthreads();
      if (*s_ok == 0) break;
      const __amdgpu_buffer_rsrc_t rR = ipc_rsrc(a.lk.rdata[gen & 1u]);
      for (int e = threadIdx.x; e < 16 * kUsN2P; e += kUsThreads) {
        const int m = e / kUsN2P, j = e - m * kUsN2P;
        sdz2[m * kUsN2P + j] =
            (m < Mi && j < N2) ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rR, (m * N2 + j) * 4, 0, 17)) : 0.f;
      }
      __syncthreads();
    } else {
    if (!us_wait(a, 8, s_ok, [&](int l, int& idx) {
          idx = kUsD + l;
          return (unsigned)(i + 1) * us_shard_n(M, l);
        }))
      break;
    {
      US_IDX();
      if (tid < 64) {
        const int m = tid >> 2, c4 = tid & 3;
        *reinterpret_cast<f32x4*>(sdl + m * kUsCP + 4 * c4) = hld4(rHB, bDL + ((par * 16 + m) * kUsCP + 4 * c4) * 4);
      }
      const int j = tid >> 2, mg = tid & 3;
      const f32x4 h = hld4(rHB, bH2 + ((par * kUsN2P + j) * 16 + 4 * mg) * 4);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) sh2[(4 * mg + jj) * kUsN2P + j] = h[jj];
    }
    __syncthreads();
    {
      US_IDX();
      const int j = tid & 127, mq = tid >> 7;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int m = 4 * mq + jj;
        float s = 0.f;
        if (j < N2)
          for (int cls = 0; cls < C; ++cls) s = fmaf(R(sdl[m * kUsCP + cls]), R(sW3[cls * N2 + j]), s);
        sdz2[m * kUsN2P + j] = sh2[m * kUsN2P + j] > 0.f ? s : 0.f;
      }
    }
    __syncthreads();
    }
    {
      US_IDX();
      const int o = tid >> 3, part = tid & 7, m = o >> 2, q = o & 3;
      float s = 0.f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) s = fmaf(R(sdz2[m * kUsN2P + part * 16 + jj]), R(sW2[q * 128 + part * 16 + jj]), s);
      s = sl_group_sum<8>(s);
      if (part == 0) sdzm[m * 4 + q] = sh1[m * 4 + q] > 0.f ? s : 0.f;
    }
    __syncthreads();
    {
      US_IDX();
      if (tid < 16) {
        const int q = tid >> 2, mg = tid & 3;
        f32x4 v;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[jj] = sdzm[(4 * mg + jj) * 4 + q];
        hst4(rHB, bDZ + ((((par * kUsRG + rg) * 128 + 4 * cc + q) * 16 + 4 * mg) * 4), v);
      }
    }
    us_arrive(a, kUsDZ + rg);
    {
      // Bob: W2[:, my rows], b1 of my rows, b2[w]; Alice: the replicated head
      US_IDX();
      {
        const int q = tid >> 7, j = tid & 127;
        if (nb + 4 * cc + q < N1 && j < N2) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g = fmaf(R(sdz2[m * kUsN2P + j]), R(sh1[m * 4 + q]), g);
          res_update<true>(a.ob, ss_b, ib_b, sW2[q * 128 + j], g, sW2[512 + q * 128 + j], sW2[1024 + q * 128 + j]);
        }
      }
      if (tid < 4 && nb + 4 * cc + tid < N1) {
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) g += sdzm[m * 4 + tid];
        res_update<true>(a.ob, ss_b, ib_b, sb1[tid], g, sb1[4 + tid], sb1[8 + tid]);
      }
      if (tid == 4 && w < N2) {
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) g += sdz2[m * kUsN2P + w];
        res_update<true>(a.ob, ss_b, ib_b, sb2[0], g, sb2[1], sb2[2]);
      }
      for (int e = tid; !REM && e < C * N2; e += kUsThreads) {
        const int cls = e / N2, j = e - cls * N2;
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) g = fmaf(R(sdl[m * kUsCP + cls]), R(sh2[m * kUsN2P + j]), g);
        res_update<true>(a.oa, ss_a, ib_a, sW3[e], g, sW3[kUsW3 + e], sW3[2 * kUsW3 + e]);
      }
      if (!REM && tid >= 32 && tid < 32 + C) {
        const int cls = tid - 32;
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) g += sdl[m * kUsCP + cls];
        res_update<true>(a.oa, ss_a, ib_a, sb3[cls], g, sb3[kUsCP + cls], sb3[2 * kUsCP + cls]);
      }
    }

    // ================= X: the row group's dz1, the cut-gradient partial from the old W1
    if (!us_wait(a, 1, s_ok, [&](int, int& idx) {
          idx = kUsDZ + rg;
          return 32u * (unsigned)(i + 1);
        }))
      break;
    {
      US_IDX();
      const int n = tid >> 2, mg = tid & 3;
      const f32x4 v = hld4(rHB, bDZ + ((((par * kUsRG + rg) * 128 + n) * 16 + 4 * mg) * 4));
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) sdz[(4 * mg + jj) * kDzP + n] = v[jj];
#pragma unroll
      for (int kb = 0; kb < kUsKB; ++kb)
        *reinterpret_cast<f32x4*>(sws + (16 * r + li) * kUsKP + 16 * kb + 4 * lq) = Wr[kb];
    }
    __syncthreads();
    {
      // wave r: column blocks r and r + 8 (< 11): dx[m][16 kb + li] = sum_n dz1[m][n] W1[n][..]
      US_IDX();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kb = r + 8 * u;
        if (kb < kUsKB) {
          f32x4 acc0 = zv, acc1 = zv;
          if constexpr (BF) {
            // n = 16 t + 4 lq + c: eight bf16 instructions over the row group's 128 rows
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const f32x4 av = *reinterpret_cast<const f32x4*>(sdz + li * kDzP + 16 * t + 4 * lq);
              f32x4 bv;
#pragma unroll
              for (int c = 0; c < 4; ++c) bv[c] = sws[(16 * t + 4 * lq + c) * kUsKP + 16 * kb + li];
              if (t & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(us_bf4(av), us_bf4(bv), acc1, 0, 0, 0);
              else acc0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(us_bf4(av), us_bf4(bv), acc0, 0, 0, 0);
              asm volatile("" ::: "memory");
            }
          } else
#pragma unroll
          for (int s = 0; s < 32; s += 2) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(sdz[li * kDzP + 4 * s + lq],
                                                        sws[(4 * s + lq) * kUsKP + 16 * kb + li], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(sdz[li * kDzP + 4 * s + 4 + lq],
                                                        sws[(4 * s + 4 + lq) * kUsKP + 16 * kb + li], acc1, 0, 0, 0);
            asm volatile("" ::: "memory");
          }
          acc0 += acc1;   // lane: dx[m = 4 lq + j][16 kb + li]
          hst4(rHB, bDX + (((((par * kUsCh + cc) * kUsRG + rg) * kUsKP + 16 * kb + li) * 16 + 4 * lq) * 4), acc0);
        }
      }
    }
    us_arrive(a, kUsDX + cc);

    if constexpr (REM) {
      // ================= (remote) the cut gradient to her, her activation of batch i + 1 in
      const int len = rows_of(i) * (kUsCh * kUsP);
      if (w < nchunks(len)) {
        if (!us_wait(a, kUsCh, s_ok, [&](int l, int& idx) {
              idx = kUsDX + l;
              return (unsigned)RG * (unsigned)(i + 1);
            }))
          break;
        const uint32_t gen = a.lk.sgen0 + 2u + 2u * (uint32_t)i;
        const int prev = i > 0 ? nchunks(rows_of(i - 1) * (kUsCh * kUsP)) : a.lk.sprev[1];
        bool sent = true;
        for (int c = w; sent && c < nchunks(len); c += G)   // 85 chunks at B = 16: more than a narrow grid
          sent = send_chunk(c, gen, prev, len, [&](int e) {
              const int m = e / (kUsCh * kUsP), k0 = e - m * (kUsCh * kUsP);
              f32x4 v;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int c = (k0 + q) / kUsP, p = (k0 + q) - c * kUsP;
                float gx = 0.f;
                for (int g = 0; g < RG; ++g)   // the row groups' partials in order, as the conv jobs
                  gx += hld1(rHB, bDX + (((((par * kUsCh + c) * kUsRG + g) * kUsKP + p) * 16 + m) * 4));
                v[q] = gx;
              }
              return v;
            });
        if (!sent) break;
      }
      if (more) {
        if (!recv_act(i + 1)) break;
        us_arrive(a, kUsXC + cc);
      }
    } else {
    // ================= C: conv job: backward, the channel's step, forward of batch i + 1
    if (!us_wait(a, 1, s_ok, [&](int, int& idx) {
          idx = kUsDX + cc;
          return 8u * (unsigned)(i + 1);
        }))
      break;
    img_put(par ^ 1, pimg);
    {
      US_IDX();
      float acc[10];
#pragma unroll
      for (int j = 0; j < 10; ++j) acc[j] = 0.f;
      if (tid < 2 * kUsP) {
        const int bl = tid / kUsP, p = tid - (tid / kUsP) * kUsP;
        const int m = 2 * rg + bl;
        if (m < M && cy > 0.f) {
          float parts[kUsRG];
#pragma unroll
          for (int g = 0; g < kUsRG; ++g)
            parts[g] = hld1(rHB, bDX + (((((par * kUsCh + cc) * kUsRG + g) * kUsKP + p) * 16 + m) * 4));
          float gx = parts[0];
#pragma unroll
          for (int g = 1; g < kUsRG; ++g) gx += parts[g];
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
      hst1(rHB, bCW + (((par * kUsCh + cc) * kUsRG + rg) * 16 + j) * 4, g);
    }
    us_arrive(a, kUsCW + cc);
    if (!us_wait(a, 1, s_ok, [&](int, int& idx) {
          idx = kUsCW + cc;
          return 8u * (unsigned)(i + 1);
        }))
      break;
    if (threadIdx.x < 10) {
      const int j = threadIdx.x;
      float parts[kUsRG];
#pragma unroll
      for (int g = 0; g < kUsRG; ++g) parts[g] = hld1(rHB, bCW + (((par * kUsCh + cc) * kUsRG + g) * 16 + j) * 4);
      float g = parts[0];
#pragma unroll
      for (int q = 1; q < kUsRG; ++q) g += parts[q];
      res_update<true>(a.oa, ss_a, ib_a, scv[j], g, scv[10 + j], scv[20 + j]);
    }
    __syncthreads();
    if (more) {
      conv_fwd(i + 1);
      us_arrive(a, kUsXC + cc);
    }
    }

    // ================= U: fc1's Adam step in registers (dW = dz1^T x_i on MFMA)
    {
      US_IDX();
#pragma unroll
      for (int kb = 0; kb < kUsKB; ++kb) {
        f32x4 g = zv;
        if constexpr (BF) {
          // the 16 batch rows m = 4 lq + c in one bf16 instruction
          f32x4 av, bv;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            av[c] = sx[(4 * lq + c) * kUsKP + 16 * kb + li];
            bv[c] = sdz[(4 * lq + c) * kDzP + 16 * r + li];
          }
          g = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(us_bf4(av), us_bf4(bv), g, 0, 0, 0);
        } else
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4)
          g = __builtin_amdgcn_mfma_f32_16x16x4f32(sx[(4 * t4 + lq) * kUsKP + 16 * kb + li],
                                                   sdz[(4 * t4 + lq) * kDzP + 16 * r + li], g, 0, 0, 0);
        // lane: dW[n = 16 r + li][16 kb + 4 lq + j] = g[j]
        res_update4<true>(a.ob, ss_b, ib_b, Wr[kb], g, Mr[kb], Vr[kb]);
        asm volatile("" ::: "memory");
      }
    }
    i_end = i + 1;
  }

fin:
  if constexpr (REM) {
    // the last step's dz2: acked once every workgroup has read it (a closing seam)
    if (i_end == a.S && a.S > 0) {
      us_arrive(a, kUsFin);
      const int s = a.S - 1;
      const uint32_t gd = a.lk.rgen0 + 2u + 2u * (uint32_t)s;
      const int nch = nchunks(rows_of(s) * N2);
      if (w < nch && us_wait(a, 1, s_ok, [&](int, int& idx) {
            idx = kUsFin;
            return (unsigned)G;
          })) {
        if (threadIdx.x == 0) ipc_raise_flag(a.lk.rack[gd & 1u] + w, gd, 0);
      }
    }
  }

  // ---- write the state back
  __syncthreads();
  {
    US_IDX();
    const int n = nb + 16 * r + li;
#pragma unroll
    for (int kb = 0; kb < kUsKB; ++kb)
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) {
        const int lc = 16 * kb + 4 * lq + comp;
        if (n < N1 && lc < kUsP) {
          const int64_t off = (int64_t)n * (kUsCh * kUsP) + kUsP * cc + lc;
          a.W1[off] = Wr[kb][comp];
          a.m1[off] = Mr[kb][comp];
          a.v1[off] = Vr[kb][comp];
        }
      }
    {
      const int q = tid >> 7, j = tid & 127, n2 = nb + 4 * cc + q;
      if (n2 < N1 && j < N2) {
        const int64_t off = (int64_t)j * N1 + n2;
        a.W2[off] = sW2[q * 128 + j];
        a.m2[off] = sW2[512 + q * 128 + j];
        a.v2[off] = sW2[1024 + q * 128 + j];
      }
    }
    if (tid < 4 && nb + 4 * cc + tid < N1) {
      const int n1 = nb + 4 * cc + tid;
      a.b1[n1] = sb1[tid];
      a.mb1[n1] = sb1[4 + tid];
      a.vb1[n1] = sb1[8 + tid];
    }
    if (tid == 0 && w < N2) {
      a.b2[w] = sb2[0];
      a.mb2[w] = sb2[1];
      a.vb2[w] = sb2[2];
    }
    if (!REM && w == 0) {
      for (int e = tid; e < C * N2; e += kUsThreads) {
        a.W3[e] = sW3[e];
        a.m3[e] = sW3[kUsW3 + e];
        a.v3[e] = sW3[2 * kUsW3 + e];
      }
      if (tid < C) {
        a.b3[tid] = sb3[tid];
        a.mb3[tid] = sb3[kUsCP + tid];
        a.vb3[tid] = sb3[2 * kUsCP + tid];
      }
    }
    if (!REM && rg == 0 && tid < 10) {
      const int j = tid;
      if (j < 9) {
        a.cw[cc * 9 + j] = scv[j];
        a.cmw[cc * 9 + j] = scv[10 + j];
        a.cvw[cc * 9 + j] = scv[20 + j];
      } else {
        a.cb[cc] = scv[9];
        a.cmb[cc] = scv[19];
        a.cvb[cc] = scv[29];
      }
    }
  }
}
#undef US_IDX

std::string ushape_check(const UsArgs& a) {
  if (a.M < 1 || a.M > 16) return "rows per step 1..16";
  if (a.rem) {
    if (a.RG != 1 && a.RG != 2 && a.RG != 4 && a.RG != 8) return "remote Alice: 1, 2, 4 or 8 row groups";
    if (a.G != 32 * a.RG || a.N1 > 128 * a.RG) return "remote Alice: 32 workgroups per 128-row group";
    if (a.N2 > a.G || a.N2 % 4) return "remote Alice: fc2 width % 4, one h2 workgroup per column";
    if (a.lk.sdata[0] == nullptr || a.lk.rdata[0] == nullptr) return "remote Alice: the channel";
  }
  if (a.N1 < 1 || a.N1 > kUsRG * 128) return "fc1 width <= 1024";
  if (a.N2 < 1 || a.N2 > kUsN2P) return "fc2 width <= 128";
  if (a.C < 1 || a.C > kUsCP || a.C * a.N2 > kUsW3) return "head classes <= 16, classes x fc2 width <= 1024";
  if (a.ob.kind != 2 || a.oa.kind != 2) return "Adam on both sides";
  if (a.S < 0) return "steps";
  return "";
}

static const void* us_kernel(const UsArgs& a) {
  if (a.rem)
    return a.bf16 ? reinterpret_cast<const void*>(&ushape_epoch_kernel<true, true>)
                  : reinterpret_cast<const void*>(&ushape_epoch_kernel<false, true>);
  return a.bf16 ? reinterpret_cast<const void*>(&ushape_epoch_kernel<true, false>)
                : reinterpret_cast<const void*>(&ushape_epoch_kernel<false, false>);
}

bool ushape_fits(const UsArgs& a, int device, std::string* why) {
  std::string s = ushape_check(a);
  if (s.empty()) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, device) != hipSuccess) {
      s = "device properties";
    } else {
      const void* fn = us_kernel(a);
      int nb = 0;
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kUsLds);
      if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kUsThreads, kUsLds);
      if (e != hipSuccess || nb < 1) s = "occupancy";
      else if ((int64_t)nb * pr.multiProcessorCount < (a.rem ? a.G : kUsG)) s = "workgroups not co-resident";
    }
  }
  if (why) *why = s;
  return s.empty();
}

hipError_t ushape_epoch_launch(const UsArgs& a, hipStream_t st) {
  if (!ushape_check(a).empty()) return hipErrorInvalidValue;
  if (a.S <= 0) return hipSuccess;
  const void* fn = us_kernel(a);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kUsLds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.cnt, 0, (size_t)kUsCounters * kUsStride * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  UsArgs arg = a;
  void* params[] = {&arg};
  const int G = a.rem ? a.G : kUsG;
  if (!a.coop) return hipLaunchKernel(fn, dim3(G), dim3(kUsThreads), params, (size_t)kUsLds, st);
  return hipLaunchCooperativeKernel(fn, dim3(G), dim3(kUsThreads), params, (unsigned)kUsLds, st);
}

}  // namespace sl
