// Register-resident server epoch: S steps of Bob's 3-layer tail in ONE persistent launch.
//
// Reference: bob.train_and_backward's inner loop (data_entities_vanilla_sisa.py:298-313),
// per cached batch `zero_grad; CE(model2_sisa(act), y).backward(); Adam.step()`, for one
// tensor-parallel shard of the tail (fc1 column-parallel, fc2 row-parallel, fc3 replicated,
// as engine/tail.py).
//
// Why: the launch-per-stage executor (engine.cpp) streams the shard's W / m / v through HBM
// (or the Infinity Cache) every step: at a TP = 8 shard ~49 MB of state, 23 us of the 52 us
// step (profiles/r3_native_step_kernels_tp1_tp8.txt).  256 CUs hold 128 MiB of VGPRs and
// 40 MiB of LDS, so a shard that narrow fits on-chip: each of the 256 workgroups (one 16-wave
// workgroup per CU) loads its slice of the state once, keeps it in registers / LDS for all S
// steps and writes it back at the end.  A step then moves only activations and hand-offs.
//
// Ownership (workgroup w of G):
//   fc1   one row block of 16 rows x up to kResTiles 256-column blocks ("tiles"): thread
//         (wave r, lane) holds W1[n0 + r][kb + 4 lane .. +3] and its m, v per tile (f32x4),
//         the input slice x_t[:, tiles] in LDS (kept from the previous step's look-ahead);
//   fc2   rows n = w + G i (i < kResRows2): wave r holds W2[n_(r/4)][q + 256 s], q = 64 (r % 4)
//         + lane; W3[:, n] and b2[n] in LDS; every workgroup keeps an identical copy of b3.
// Step t, four in-launch hand-offs ("seams", each: write-through (sc1) payload stores, every
// wave drains, one agent-scope counter add per workgroup on a per-XCD shard; consumers poll
// the shards, then read with sc1 loads — MI355X_MICROARCH.md, the valid-forms table row 1):
//   [A]  each fc1 row block's last-arriving column group summed the groups' look-ahead
//        partials of x_t W1_t^T (+ b1_t) and published h1_t = drop(relu(.)); every workgroup
//        reads h1_t into LDS, then its fc2
//        rows' product P2[:, n] = h1 W2[n, :]^T (tensor-parallel: the peer-mapped exchange of
//        those rows with the other ranks, summed in rank order), h2 = drop(relu(P2 + b2)) and
//        its share of the logits, sum_n h2[:, n] W3[:, n]^T;
//   [B]  workgroup m < M sums row m's 256 logit partials + b3, softmax-CE, dlogits row m;
//   [C]  every workgroup: b3's Adam step; for its fc2 rows dh2 = dlog W3[:, n], dz2 (ReLU /
//        dropout mask), W3 / b2 / W2 Adam steps; publishes dz2[:, n] and W2_{t+1}[n, :];
//   [D]  fc1 workgroups: dz1 for their 16 rows = dz2 W2_t[:, rows] (MFMA over the 1000 fc2
//        rows, W2_t from the previous step's publication), ReLU / dropout mask, b1 / W1
//        Adam steps in registers, and the next batch's look-ahead product with W1_{t+1}
//        (exact-fp32 MFMA over the tile, as wgrad_group_kernel) -> seam A of step t + 1.
// Arithmetic is fp32 throughout (exact-fp32 MFMA for the two products that use it); the sums
// are in fixed orders, so a run is deterministic; the summation order differs from the
// launch-per-stage executor's, so results agree with it (and with torch) to fp32 rounding,
// not bitwise (tests/test_resident_gpu.py).
//
// Safety: every wait is bounded (wall clock; a timeout raises a[.err] and every other wait
// then gives up at once), so a stuck launch ends.  The workgroups wait on each other, so all G
// must be resident at once: the host checks the occupancy of the instantiation it launches
// (resident_fits) and launches cooperatively (hipLaunchCooperativeKernel refuses a grid the
// device cannot hold at once instead of queueing part of it).  Nothing else may occupy the
// device's CUs during the launch (the SISA server phase runs no other stream on Bob's GPU).
#include "resident.h"
#include "persist.h"

#include <string>

namespace sl {

namespace {

using namespace persist;

// Publish this workgroup's hand-off stores of `seam`: every wave drains its (write-through)
// stores, the barrier orders all the drains before thread 0's counter add.
__device__ __forceinline__ void arrive(unsigned* cnt, int seam, int w) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(cnt + (seam * 8 + (w & 7)) * kResShardStride, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Row-block hand-off (fc1 look-ahead partials of one 16-row block's column groups to the
// block's last-arriving group): one counter per row block after the seam shards.
__device__ __forceinline__ unsigned* rb_counter(unsigned* cnt, int rb) {
  return cnt + (kResSeams * 8 + rb) * kResShardStride;
}

// Wait until every shard of `seam` holds `mult` arrivals per producer of that shard (lanes
// 0..7 of wave 0 poll one shard each, relaxed, with s_sleep); the barrier then releases every
// wave to its sc1 loads.  False (uniform over the workgroup) when the wait gave up.
__device__ __forceinline__ bool seam_wait(const ResArgs& a, int seam, unsigned mult, int* s_ok) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < 8) {
      const int n = a.shard_n[seam * 8 + lane];
      const unsigned* p = a.cnt + (seam * 8 + lane) * kResShardStride;
      const unsigned tgt = mult == 0xffffffffu ? mult : mult * (unsigned)n;   // ~0u: never met
      if (n > 0 && poll(p) < tgt) {
        const uint64_t t0 = wall_clock64();
        while (poll(p) < tgt) {
          if (failed(a.err)) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if ((int64_t)(wall_clock64() - t0) > a.timeout) {
            __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = false;
            break;
          }
        }
      }
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return *s_ok != 0;
}

// LDS carve (bytes; every offset a multiple of 16)
constexpr int kSxBytes = 16 * kResTiles * 256 * 4;   // x_t slice of the fc1 tiles
constexpr int kSh1Max = 768;                         // N1p bound (6 W2 slots of 128 per thread)
constexpr int OFF_SX = 0;
constexpr int OFF_SH1 = OFF_SX + kSxBytes;            // h1 [16][N1p]; look-ahead staging aliases it
constexpr int OFF_RED = OFF_SH1 + 16 * kSh1Max * 4;   // [8][64] f32x4 / logits [16][32] f32x4
static_assert(2 * 16 * 65 * 16 <= 16 * kSh1Max * 4, "two staged look-ahead tiles fit the h1 region");
constexpr int OFF_SDZ = OFF_RED + 8 * 64 * 16;        // dz1 [16][16]
constexpr int OFF_SDL = OFF_SDZ + 16 * 16 * 4;        // dlogits [16][kResMaxC]
constexpr int OFF_SH2 = OFF_SDL + 16 * kResMaxC * 4;  // h2 [16][4]
constexpr int OFF_SDZ2 = OFF_SH2 + 16 * 4 * 4;        // dz2 [16][4]
constexpr int OFF_RED2 = OFF_SDZ2 + 16 * 4 * 4;       // fc2 row sums [8 waves][16]
constexpr int OFF_W3 = OFF_RED2 + 16 * 16 * 4;        // W3 columns {W, m, v}[4][kResMaxC]
constexpr int OFF_B3 = OFF_W3 + 3 * 4 * kResMaxC * 4; // b3 {W, m, v}[kResMaxC]
constexpr int OFF_B2 = OFF_B3 + 3 * kResMaxC * 4;     // b2 {W, m, v}[4]
constexpr int OFF_B1 = OFF_B2 + 3 * 4 * 4;            // b1 {W, m, v}[16]
constexpr int OFF_W2N = OFF_B1 + 3 * 16 * 4;         // W2 after the step, [4 rows][kSh1Max] (publication)
constexpr int OFF_OK = OFF_W2N + 4 * kSh1Max * 4;
constexpr int kResLds = OFF_OK + 16;

}  // namespace

// Per-lane indices, re-derived from a laundered thread id at the top of every phase: the
// compiler then recomputes the addresses built on them where they are used instead of
// holding them (and everything derived from them) in VGPRs across the whole step loop, which
// the state-holding registers cannot afford (measured: ~110 VGPRs of spills without it).
// Thread (wave r of 8, lane): fc1 rows n0 + r and n0 + r + 8 of every tile; fc2 row slot
// r / 2, W2 columns q2 + 128 s.
#define RES_IDX()                                                        \
  int tid_l_ = threadIdx.x;                                              \
  asm volatile("" : "+v"(tid_l_));                                       \
  const int tid = tid_l_, r = tid >> 6, lane = tid & 63, li = lane & 15, lq = lane >> 4; \
  const int n1 = n0 + r, i2 = r >> 1, n2 = w + G * i2;                   \
  const bool own2 = n2 < N2;                                             \
  const int q2 = ((r & 1) << 6) | lane;                                  \
  (void)li; (void)lq; (void)n1; (void)own2; (void)q2

// phase timestamp k of step i (workgroups 0 and G - 1, thread 0; off unless a.trace is set)
#define RES_MARK(k)                                                                              \
  do {                                                                                           \
    if (a.trace != nullptr && i < a.trace_steps && threadIdx.x == 0 && (w == 0 || w == G - 1))  \
      a.trace[((int64_t)(w == 0 ? 0 : 1) * a.trace_steps + i) * 16 + (k)] = (int64_t)wall_clock64(); \
  } while (0)

template <bool ADAM>
__global__ void __launch_bounds__(kResThreads) resident_epoch_kernel(ResArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x4* sx = reinterpret_cast<f32x4*>(smem + OFF_SX);     // [16][kResTiles * 64]
  float* sh1 = reinterpret_cast<float*>(smem + OFF_SH1);   // [16][SH1P]
  f32x4* sw = reinterpret_cast<f32x4*>(smem + OFF_SH1);    // [16][65] (look-ahead staging)
  f32x4* red = reinterpret_cast<f32x4*>(smem + OFF_RED);
  float* sdz = reinterpret_cast<float*>(smem + OFF_SDZ);
  float* sdl = reinterpret_cast<float*>(smem + OFF_SDL);
  float* sh2 = reinterpret_cast<float*>(smem + OFF_SH2);
  float* sdz2 = reinterpret_cast<float*>(smem + OFF_SDZ2);
  float* red2 = reinterpret_cast<float*>(smem + OFF_RED2);
  float* sW3 = reinterpret_cast<float*>(smem + OFF_W3);
  float* sb3 = reinterpret_cast<float*>(smem + OFF_B3);
  float* sb2 = reinterpret_cast<float*>(smem + OFF_B2);
  float* sb1 = reinterpret_cast<float*>(smem + OFF_B1);
  float* sW2n = reinterpret_cast<float*>(smem + OFF_W2N);
  int* s_ok = reinterpret_cast<int*>(smem + OFF_OK);
  constexpr int NW = kResThreads / 64;                      // 8 waves
  constexpr int XS = kResTiles * 64;                        // sx row pitch (f32x4)
  constexpr int MC = kResMaxC;
  constexpr int SH1P = kSh1Max;                             // h1 row pitch (floats)
  constexpr int S2 = kSh1Max / 128;                         // W2 slots per thread

  const int w = blockIdx.x;
  const int M = a.M, N1 = a.N1, N1p = a.N1p, K1 = a.K1, N2 = a.N2, C = a.C, C4 = a.C4, G = a.G;
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};

  // ---- roles (workgroup-uniform)
  const bool fc1 = w < a.nfc1;
  const int rb = fc1 ? w / a.ngrp : 0;
  const int grp = fc1 ? w - rb * a.ngrp : 0;
  const int n0 = rb * 16, cb0 = grp * kResTiles;
  const int nct = fc1 ? min(kResTiles, a.ncb - cb0) : 0;
  const __amdgpu_buffer_rsrc_t rLA = rs_of(a.LA), rH1 = rs_of(a.H1), rLP = rs_of(a.LP), rDL = rs_of(a.DL),
                               rDZ = rs_of(a.DZ2), rW2B = rs_of(a.W2B);

  // ---- load the state: fc1 rows n1 + 8 h of tile ct in p / s0 / s1[ct][h]
  f32x4 p[kResTiles][2], s0[kResTiles][2], s1[kResTiles][2];
  float w2[S2], w2m[S2], w2v[S2];
  {
    RES_IDX();
#pragma unroll
    for (int ct = 0; ct < kResTiles; ++ct)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        p[ct][h] = s0[ct][h] = s1[ct][h] = zv;
        const int k = (cb0 + ct) * 256 + 4 * lane, n = n1 + 8 * h;
        if (ct < nct && n < N1 && k < K1) {
          const int64_t off = (int64_t)n * K1 + k;
          p[ct][h] = *reinterpret_cast<const f32x4*>(a.L1.W + off);
          s0[ct][h] = *reinterpret_cast<const f32x4*>(a.L1.m + off);
          if (ADAM) s1[ct][h] = *reinterpret_cast<const f32x4*>(a.L1.v + off);
        }
      }
#pragma unroll
    for (int s = 0; s < S2; ++s) {
      w2[s] = w2m[s] = w2v[s] = 0.f;
      const int j = q2 + 128 * s;
      if (own2 && j < N1) {
        const int64_t off = (int64_t)n2 * N1 + j;
        w2[s] = a.L2.W[off];
        w2m[s] = a.L2.m[off];
        if (ADAM) w2v[s] = a.L2.v[off];
      }
    }
    if (tid < 4 * MC) {
      const int ii = tid / MC, c = tid - ii * MC;
      const int n = w + G * ii;
      const bool ok = n < N2 && c < C;
      const int64_t off = (int64_t)c * N2 + n;
      sW3[(0 * 4 + ii) * MC + c] = ok ? a.L3.W[off] : 0.f;
      sW3[(1 * 4 + ii) * MC + c] = ok ? a.L3.m[off] : 0.f;
      sW3[(2 * 4 + ii) * MC + c] = (ok && ADAM) ? a.L3.v[off] : 0.f;
    }
    if (tid < MC) {
      const bool ok = tid < C;
      sb3[tid] = ok ? a.L3.b[tid] : 0.f;
      sb3[MC + tid] = ok ? a.L3.mb[tid] : 0.f;
      sb3[2 * MC + tid] = (ok && ADAM) ? a.L3.vb[tid] : 0.f;
    }
    if (tid < 4) {
      const int n = w + G * tid;
      const bool ok = n < N2;
      sb2[tid] = ok ? a.L2.b[n] : 0.f;
      sb2[4 + tid] = ok ? a.L2.mb[n] : 0.f;
      sb2[8 + tid] = (ok && ADAM) ? a.L2.vb[n] : 0.f;
    }
    if (tid < 16) {
      const int n = n0 + tid;
      const bool ok = fc1 && grp == 0 && n < N1;
      sb1[tid] = ok ? a.L1.b[n] : 0.f;
      sb1[16 + tid] = ok ? a.L1.mb[n] : 0.f;
      sb1[32 + tid] = (ok && ADAM) ? a.L1.vb[n] : 0.f;
    }
  }

  // a batch's input slice in MFMA A layout: lane (li, lq) of wave r holds, for column group
  // h, x[row li][kb + 16 (r + 8 h) + 4 lq .. +3] of tile ct (rows >= M read as 0)
  auto load_x = [&](int batch, f32x4 (&xv)[kResTiles][2], int ct0 = 0, int ct1 = kResTiles) {
    RES_IDX();
#pragma unroll
    for (int ct = 0; ct < kResTiles; ++ct)
      if (ct >= ct0 && ct < ct1)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = (cb0 + ct) * 256 + 16 * (r + 8 * h) + 4 * lq;
        xv[ct][h] = (ct < nct && li < M && k < K1)
                        ? *reinterpret_cast<const f32x4*>(a.X + ((int64_t)batch * M + li) * K1 + k)
                        : zv;
      }
  };
  // ... kept in LDS as the next step's x_t (row li, float4 column 16 (r + 8 h) + 4 lq of tile ct)
  auto stash_x = [&](const f32x4 (&xv)[kResTiles][2]) {
    RES_IDX();
#pragma unroll
    for (int ct = 0; ct < kResTiles; ++ct)
#pragma unroll
      for (int h = 0; h < 2; ++h) sx[li * XS + ct * 64 + 4 * (r + 8 * h) + lq] = xv[ct][h];
  };
  // the look-ahead: pre[m][n0 + nn] = sum over this workgroup's columns of x[m] . W1[n0 + nn]
  // (exact-fp32 MFMA 16x16x4; the updated tile staged through LDS into B layout, rows padded
  // to 65 float4, as wgrad_group_kernel; wave r covers the tile's 16-column groups r and
  // r + 8) -> LA[par][grp]; the row block's last-arriving column group turns the groups'
  // partials into h1 rows (H1[par]) for step `step` and publishes them (seam A).  (Returns
  // true: no wait in it can give up.)
  auto lookahead = [&](const f32x4 (&xv)[kResTiles][2], int par, int step, unsigned mult) -> bool {
    RES_IDX();
    f32x4 z = zv;
#pragma unroll
    for (int ct0 = 0; ct0 < kResTiles; ct0 += 2) {       // two tiles staged per barrier pair
      if (ct0 < nct) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int ct = ct0 + u, k = (cb0 + ct) * 256 + 4 * lane;
#pragma unroll
          for (int h = 0; h < 2; ++h)
            sw[u * 16 * 65 + (r + 8 * h) * 65 + lane] = (ct < nct && n1 + 8 * h < N1 && k < K1) ? p[ct][h] : zv;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int ct = ct0 + u;
          if (ct < nct) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f32x4 wv4 = sw[u * 16 * 65 + li * 65 + 4 * (r + 8 * h) + lq];
#pragma unroll
              for (int c = 0; c < 4; ++c)
                z = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[ct][h][c], wv4[c], z, 0, 0, 0);
            }
          }
        }
        __syncthreads();
      }
    }
    red[r * 64 + lane] = z;   // z[j] = partial(m = 4 lq + j, n = n0 + li)
    __syncthreads();
    // every column group publishes its partial (group 0's with b1 added: it holds the bias);
    // the row block's LAST arriver (the returning counter add tells it) sums the ngrp partials
    // in group order, applies ReLU and dropout (the consuming step's seed), publishes h1 rows
    // [n0, n0 + 16) and arrives at seam A.  No workgroup waits: a fixed reducer (group 0)
    // polled for the other groups, 0.5-1 us of the step.
    if (tid < 256) {
      const int m = tid >> 4, nn = tid & 15;
      float own = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) own += red[ww * 64 + 16 * (m >> 2) + nn][m & 3];
      if (grp == 0) own += sb1[nn];
      if (m < M && n0 + nn < N1) hst1(rLA, ((((par * a.ngrp + grp) * 16) + m) * N1p + n0 + nn) * 4, own);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(rb_counter(a.cnt, rb), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_ok = (old == (unsigned)a.ngrp * mult - 1u) ? 1 : 0;
    }
    __syncthreads();
    if (*s_ok == 0) return true;
    if (tid < 256) {
      const int m = tid >> 4, nn = tid & 15, n = n0 + nn;
      if (m < M && n < N1) {
        float parts[kResGroups];
#pragma unroll
        for (int g = 0; g < kResGroups; ++g)
          parts[g] = g < a.ngrp ? hld1(rLA, ((((par * a.ngrp + g) * 16) + m) * N1p + n) * 4) : 0.f;
        float v = parts[0];
#pragma unroll
        for (int g = 1; g < kResGroups; ++g) v += parts[g];
        v = drop_relu(v, a.seeds[4 * step], a.seeds[4 * step + 1], m, a.col_off1 + n, a.thr1, a.dsc1);
        hst1(rH1, ((par * 16 + m) * N1p + n) * 4, v);
      }
    }
    arrive(a.cnt, 0, rb);            // seam A's shards count row blocks (rb % 8)
    return true;
  };
  // W2 after a step, in the fc1 tiles' layout W2B[par][rb(j)][w][j % 16][ii] (this workgroup's
  // four rows n = w + G ii side by side: gathered through LDS, one float4 store per column)
  auto publish_w2 = [&](int par) {
    {
      RES_IDX();
#pragma unroll
      for (int s = 0; s < S2; ++s) {
        const int j = q2 + 128 * s;
        if (j < N1) sW2n[i2 * kSh1Max + j] = own2 ? w2[s] : 0.f;
      }
    }
    __syncthreads();
    {
      RES_IDX();
      for (int j = tid; j < N1; j += kResThreads) {
        const f32x4 v = {sW2n[j], sW2n[kSh1Max + j], sW2n[2 * kSh1Max + j], sW2n[3 * kSh1Max + j]};
        hst4(rW2B, ((((par * a.nrb + (j >> 4)) * G + w) * 16 + (j & 15)) * 4) * 4, v);
      }
    }
  };

  // ---- prologue: W2_0 for the first step's dz1; the first batch's look-ahead -> seam A (step 0)
  publish_w2(0);
  bool fc1_failed = false;
  if (fc1) {
    f32x4 xv[kResTiles][2];
    load_x(0, xv);
    stash_x(xv);
    if (!lookahead(xv, 0, 0, 1u)) fc1_failed = true;
  }

  for (int i = 0; i < a.S && !fc1_failed; ++i) {
    const int par = i & 1, nxt = par ^ 1;
    const uint32_t sd2 = a.seeds[4 * i + 2], sd3 = a.seeds[4 * i + 3];
    const SlOpt o = a.o;
    float ss = ADAM ? a.adam[4 * i] : 0.f, ib = ADAM ? a.adam[4 * i + 1] : 0.f;
    asm volatile("" : "+v"(ss), "+v"(ib));   // held in VGPRs (res_update)

    // ================= A: h1_t, fc2 rows, logit partials
    RES_MARK(0);
    // fault injection (tests): at step fault_step this wait cannot be met, times out (err 2) and
    // every other wait gives up, as a hand-off that never arrives would make them
    if (!seam_wait(a, 0, i == a.fault_step ? 0xffffffffu : (unsigned)(i + 1), s_ok)) break;
    RES_MARK(1);
    {
      RES_IDX();
      // h1_t rows as published by each row block's last-arriving column group (rows >= M are zero)
      const int q4 = N1p >> 2;
      constexpr int U = (16 * kSh1Max / 4 + kResThreads - 1) / kResThreads;   // float4 per thread
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = tid + u * kResThreads;
        const int m = e / q4, j = 4 * (e - m * q4);
        v[u] = (e < 16 * q4 && m < M) ? hld4(rH1, ((par * 16 + m) * N1p + j) * 4) : zv;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = tid + u * kResThreads;
        const int m = e / q4, j = 4 * (e - m * q4);
        if (e < 16 * q4) *reinterpret_cast<f32x4*>(sh1 + m * SH1P + j) = v[u];
      }
    }
    __syncthreads();
    RES_MARK(2);
    {
      // this wave's fc2 row: 16 partial sums over its W2 slots, then wave sums
      RES_IDX();
      float acc[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) acc[m] = 0.f;
#pragma unroll
      for (int s = 0; s < S2; ++s) {
        const int j = q2 + 128 * s;
        if (own2 && j < N1) {
#pragma unroll
          for (int m = 0; m < 16; ++m) acc[m] = fmaf(sh1[m * SH1P + j], w2[s], acc[m]);
        }
      }
      // the 16 wave sums as one reduce-scatter: each exchange halves the values a lane holds
      // (17 lane exchanges instead of 16 x 6); lane L ends with row m = L[5:2]
#pragma unroll
      for (int h = 8, bit = 32; h >= 1; h >>= 1, bit >>= 1) {
        const bool up = (lane & bit) != 0;
#pragma unroll
        for (int u = 0; u < h; ++u) {
          const float keep = up ? acc[h + u] : acc[u], send = up ? acc[u] : acc[h + u];
          acc[u] = keep + __shfl_xor(send, bit);
        }
      }
      float t = acc[0];
      t += __shfl_xor(t, 2);
      t += __shfl_xor(t, 1);
      if ((lane & 3) == 0) red2[r * 16 + (lane >> 2)] = t;
    }
    __syncthreads();
    RES_MARK(3);
    {
      RES_IDX();
      if (tid < 64) {
        // P2[m][ii]: the two waves of row slot ii, in order
        const int m = tid >> 2, ii = tid & 3;
        float pv = red2[(2 * ii) * 16 + m] + red2[(2 * ii + 1) * 16 + m];
        if (a.ipc.T > 0) {
          // tensor-parallel fc2: this workgroup's 16 x 4 product block to every rank as 8-byte
          // granules {tag = step generation, value} (one untorn system-scope store each: the
          // data is its own flag, no flag word and no fences), polled by the receiving lane
          // until every source's tag matches, then summed in rank order (bitwise the same sum
          // on every rank).  Region reuse is ordered by the exchange itself: a rank sends step
          // i only after it received every rank's step i - 1, i.e. after each receiver finished
          // reading the slot's previous use (step i - 2, same parity).
          const uint32_t gen = a.ipc.gen + (uint32_t)i;
          const int ipar = (int)(gen & 1u), T = a.ipc.T, me = a.ipc.me;
          const int64_t half = a.ipc.cap >> 1;                   // granules per (parity, source)
          const int64_t slot = (int64_t)w * 64 + tid;
          const uint64_t gr = ((uint64_t)gen << 32) | (uint64_t)__builtin_bit_cast(uint32_t, pv);
          for (int rr = 0; rr < T; ++rr)
            __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ipc.P.data[rr]) + (ipar * T + me) * half + slot, gr,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const uint64_t* mine = reinterpret_cast<const uint64_t*>(a.ipc.P.data[me]);
          bool ok = true;
          float sum = 0.f;
          for (int src = 0; src < T && ok; ++src) {
            const uint64_t* g = mine + (ipar * T + src) * half + slot;
            uint64_t x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((uint32_t)(x >> 32) != gen) {
              const uint64_t t0 = wall_clock64();
              while ((uint32_t)((x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >> 32) != gen) {
                if (__hip_atomic_load(a.ipc.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                  ok = false;
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
                if ((int64_t)(wall_clock64() - t0) > a.ipc.timeout) {
                  ipc_fail(a.ipc.err, a.ipc.herr);
                  ok = false;
                  break;
                }
              }
            }
            sum += __builtin_bit_cast(float, (uint32_t)(x & 0xffffffffull));
          }
          ok = __all(ok);
          if (!ok && tid == 0) __hip_atomic_fetch_or(a.err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          pv = sum;
          if (tid == 0) *s_ok = ok ? 1 : 0;
        }
        const int n = w + G * ii;
        float h = 0.f;
        if (m < M && n < N2) h = drop_relu(pv + sb2[ii], sd2, sd3, m, n, a.thr2, a.dsc2);
        sh2[m * 4 + ii] = h;
      }
    }
    __syncthreads();
    if (a.ipc.T > 0 && *s_ok == 0) break;
    RES_MARK(4);
    {
      // logit partials of this workgroup's fc2 rows: LP[par][w][m][c] = sum_ii h2[m][ii] W3[c][n_ii]
      RES_IDX();
      const int nc4 = C4 >> 2;
      if (tid < 16 * nc4) {
        const int m = tid / nc4, c = 4 * (tid - m * nc4);
        if (m < M) {
          f32x4 v = zv;
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) v += sh2[m * 4 + ii] * *reinterpret_cast<const f32x4*>(sW3 + ii * MC + c);
          hst4(rLP, (((par * G + w) * 16 + m) * C4 + c) * 4, v);
        }
      }
    }
    arrive(a.cnt, 1, w);
    RES_MARK(5);

    // ================= B: row m's logits, softmax-CE, dlogits (workgroups m < M)
    if (w < M) {
      if (!seam_wait(a, 1, (unsigned)(i + 1), s_ok)) break;
      RES_MARK(6);
      RES_IDX();
      const int m = w;
      const int nc4 = C4 >> 2;
      constexpr int NG = kResThreads / 32;                  // 16 partial-sum groups
      {
        const int c4 = tid & 31, gq = tid >> 5;
        f32x4 v = zv;
        if (c4 < nc4) {
          f32x4 parts[256 / NG];
#pragma unroll
          for (int k = 0; k < 256 / NG; ++k) {
            const int src = gq + NG * k;
            parts[k] = src < G ? hld4(rLP, (((par * G + src) * 16 + m) * C4 + 4 * c4) * 4) : zv;
          }
#pragma unroll
          for (int k = 0; k < 256 / NG; ++k) v += parts[k];
        }
        red[gq * 32 + c4] = v;
      }
      __syncthreads();
      if (tid < 64) {
        const int c4 = tid & 31;
        const bool act = tid < 32 && c4 < nc4;
        f32x4 lg = zv;
        if (act) {
#pragma unroll
          for (int gq = 0; gq < NG; ++gq) lg += red[gq * 32 + c4];
          lg += *reinterpret_cast<const f32x4*>(sb3 + 4 * c4);
        }
        const int64_t lab = a.Y[(int64_t)i * M + m];
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
          const int cc = 4 * c4 + c;
          if (act && cc < C) {
            e[c] = expf(lg[c] - mx);
            se += e[c];
            if (cc == lab) zl = lg[c];
          }
        }
        se = sl_wave_sum(se);
        zl = sl_wave_sum(zl);
        const float inv = 1.f / se;
        f32x4 d = zv;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int cc = 4 * c4 + c;
          float pr = e[c] * inv;
          if (cc == lab) pr -= 1.f;
          d[c] = (ign || cc >= C) ? 0.f : pr * a.adam[4 * i + 2];
        }
        if (act) hst4(rDL, ((par * 16 + m) * C4 + 4 * c4) * 4, d);
        if (tid == 0) a.loss[(int64_t)i * M + m] = ign ? 0.f : mx + logf(se) - zl;
      }
      arrive(a.cnt, 2, w);
      RES_MARK(7);
    }

    // ================= C: b3; dz2, W3 / b2 / W2 steps of this workgroup's fc2 rows
    if (!seam_wait(a, 2, (unsigned)(i + 1), s_ok)) break;
    RES_MARK(8);
    {
      RES_IDX();
      const int nc4 = C4 >> 2;
      if (tid < 16 * nc4) {
        const int m = tid / nc4, c = 4 * (tid - m * nc4);
        *reinterpret_cast<f32x4*>(sdl + m * MC + c) = m < M ? hld4(rDL, ((par * 16 + m) * C4 + c) * 4) : zv;
      }
    }
    __syncthreads();
    {
      // dh2[m][ii] = sum_c dlog[m][c] W3[c][n_ii] (old W3): 16 lanes per (m, ii)
      RES_IDX();
#pragma unroll
      for (int oi0 = 0; oi0 < 64; oi0 += kResThreads / 16) {
        const int oi = oi0 + (tid >> 4), part = tid & 15;
        const int m = oi >> 2, ii = oi & 3;
        float s = 0.f;
#pragma unroll
        for (int c0 = 0; c0 < MC; c0 += 16) {   // classes >= C hold zeros
          const int c = c0 + part;
          s = fmaf(sdl[m * MC + c], sW3[ii * MC + c], s);
        }
        s = sl_row16_sum(s);
        if (part == 0) {
          const float h = sh2[m * 4 + ii];
          sdz2[m * 4 + ii] = (m < M && h > 0.f) ? s * a.dsc2 : 0.f;
        }
      }
    }
    __syncthreads();
    {
      RES_IDX();
      if (tid < M)   // DZ2[par][m][w][ii] = dz2[m][n = w + G ii]
        hst4(rDZ, (((par * 16 + tid) * G + w) * 4) * 4, *reinterpret_cast<const f32x4*>(sdz2 + tid * 4));
    }
    arrive(a.cnt, 3, w);
    RES_MARK(9);
    // the optimizer steps of b3, W3, b2 and W2 and W2_{t+1}'s publication (for the next step's
    // dz1) after the seam: only dz2 is on its critical path; they fill this workgroup's wait
    // for the other workgroups' dz2 (the next step's seam-B arrival drains the W2 stores, long
    // before its seam D releases their readers)
    {
      RES_IDX();
      if (tid < C) {
        // b3: identical on every workgroup
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) g += sdl[m * MC + tid];   // rows >= M are zero
        res_update<ADAM>(o, ss, ib, sb3[tid], g, sb3[MC + tid], sb3[2 * MC + tid]);
      }
      for (int e = tid; e < 4 * MC; e += kResThreads) {
        const int ii = e / MC, c = e - ii * MC;
        if (c < C && w + G * ii < N2) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g = fmaf(sdl[m * MC + c], sh2[m * 4 + ii], g);
          res_update<ADAM>(o, ss, ib, sW3[ii * MC + c], g, sW3[(4 + ii) * MC + c], sW3[(8 + ii) * MC + c]);
        }
      }
      if (tid < 4 && w + G * tid < N2) {
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) g += sdz2[m * 4 + tid];
        res_update<ADAM>(o, ss, ib, sb2[tid], g, sb2[4 + tid], sb2[8 + tid]);
      }
#pragma unroll
      for (int s = 0; s < S2; ++s) {
        const int j = q2 + 128 * s;
        if (own2 && j < N1) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g = fmaf(sdz2[m * 4 + i2], sh1[m * SH1P + j], g);
          res_update<ADAM>(o, ss, ib, w2[s], g, w2m[s], w2v[s]);
        }
      }
    }
    RES_MARK(14);
    // W2_{t+1}'s publication: fc1 workgroups issue it after their dz1 (its write-through stores
    // ahead of seam D's poll held the poll until they were acknowledged: 2.7 us measured)
    if (!fc1) publish_w2(nxt);
    RES_MARK(15);

    // ================= D: fc1 rows' dz1, b1 / W1 steps, next batch's look-ahead
    if (fc1) {
      const bool more = i + 1 < a.S;
      // dz1[m][nn] = sum_n dz2[m][n] W2_t[n][n0 + nn]; fc2 rows in the publishers' order: block
      // b = 4 workgroups w' = 4 b + lq, MFMA k index c = ii, i.e. n = w' + G c.  The seam is
      // polled with no loads in flight (the updates above have filled the wait, so it passes in
      // one poll: issued behind W2_t's operand loads it waited for them, measured 4.3 us from
      // the publication to the release), then both operands load in one round trip.
      constexpr int KB = 256 / 4 / NW;                       // blocks per wave (G <= 256)
      if (!seam_wait(a, 3, (unsigned)(i + 1), s_ok)) break;
      RES_MARK(10);
      {
        RES_IDX();
        f32x4 acc = zv;
        f32x4 A4[KB], B4[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const int wp = 4 * (r + NW * k) + lq;
          B4[k] = (wp < G && n0 + li < N1) ? hld4(rW2B, ((((par * a.nrb + rb) * G + wp) * 16 + li) * 4) * 4) : zv;
          A4[k] = (wp < G && li < M) ? hld4(rDZ, (((par * 16 + li) * G + wp) * 4) * 4) : zv;
        }
#pragma unroll
        for (int k = 0; k < KB; k += 2) {   // two chains: consecutive MFMAs independent
          f32x4 acc1 = zv;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A4[k][c], B4[k][c], acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A4[k + 1][c], B4[k + 1][c], acc1, 0, 0, 0);
          }
          acc += acc1;
        }
        red[r * 64 + lane] = acc;
      }
      __syncthreads();
      {
        RES_IDX();
        if (tid < 256) {
          const int m = tid >> 4, nn = tid & 15;
          float v = 0.f;
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) v += red[ww * 64 + 16 * (m >> 2) + nn][m & 3];
          const int n = n0 + nn;
          const bool keep = m < M && n < N1 && sh1[m * SH1P + n] > 0.f;
          sdz[m * 16 + nn] = keep ? v * a.dsc1 : 0.f;
        }
      }
      __syncthreads();
      publish_w2(nxt);
      RES_MARK(11);
      // the next batch's inputs: the first two tiles' loads issued under the dW / Adam work
      // below, the rest after it (all four up front spill the state registers)
      f32x4 xv[kResTiles][2];
      if (more) load_x(i + 1, xv, 0, 2);
      {
        RES_IDX();
        if (grp == 0 && tid < 16 && n0 + tid < N1) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdz[m * 16 + tid];
          res_update<ADAM>(o, ss, ib, sb1[tid], g, sb1[16 + tid], sb1[32 + tid]);
        }
#pragma unroll
        for (int ct = 0; ct < kResTiles; ++ct) {
          const int k = (cb0 + ct) * 256 + 4 * lane;
          if (ct < nct && k < K1) {
            // dW of rows n1 and n1 + 8 = sum_m dz1[m][row] x[m][cols] (one LDS read of x per
            // m serves both rows)
            f32x4 g0 = zv, g1 = zv;
#pragma unroll
            for (int m = 0; m < 16; ++m) {
              const f32x4 xm = sx[m * XS + ct * 64 + lane];
              g0 += sdz[m * 16 + r] * xm;
              g1 += sdz[m * 16 + r + 8] * xm;
            }
            if (n1 < N1) res_update4<ADAM>(o, ss, ib, p[ct][0], g0, s0[ct][0], s1[ct][0]);
            if (n1 + 8 < N1) res_update4<ADAM>(o, ss, ib, p[ct][1], g1, s0[ct][1], s1[ct][1]);
          }
        }
      }
      RES_MARK(12);
      if (more) {
        // the LDS copy of the next batch's inputs for the next step's dW goes in after the
        // look-ahead (its barriers also order every wave's dW reads of x_t before the overwrite)
        load_x(i + 1, xv, 2, kResTiles);
        const bool ok = lookahead(xv, nxt, i + 1, (unsigned)(i + 2));
        stash_x(xv);
        if (!ok) break;
        RES_MARK(13);
      }
    }
  }

  // ---- write the state back
  {
    RES_IDX();
#pragma unroll
    for (int ct = 0; ct < kResTiles; ++ct)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = (cb0 + ct) * 256 + 4 * lane, n = n1 + 8 * h;
        if (ct < nct && n < N1 && k < K1) {
          const int64_t off = (int64_t)n * K1 + k;
          *reinterpret_cast<f32x4*>(a.L1.W + off) = p[ct][h];
          *reinterpret_cast<f32x4*>(a.L1.m + off) = s0[ct][h];
          if (ADAM) *reinterpret_cast<f32x4*>(a.L1.v + off) = s1[ct][h];
        }
      }
#pragma unroll
    for (int s = 0; s < S2; ++s) {
      const int j = q2 + 128 * s;
      if (own2 && j < N1) {
        const int64_t off = (int64_t)n2 * N1 + j;
        a.L2.W[off] = w2[s];
        a.L2.m[off] = w2m[s];
        if (ADAM) a.L2.v[off] = w2v[s];
      }
    }
  }
  __syncthreads();
  {
    RES_IDX();
    for (int e = tid; e < 4 * MC; e += kResThreads) {
      const int ii = e / MC, c = e - ii * MC;
      const int n = w + G * ii;
      if (n < N2 && c < C) {
        const int64_t off = (int64_t)c * N2 + n;
        a.L3.W[off] = sW3[ii * MC + c];
        a.L3.m[off] = sW3[(4 + ii) * MC + c];
        if (ADAM) a.L3.v[off] = sW3[(8 + ii) * MC + c];
      }
    }
    if (w == 0 && tid < C) {
      a.L3.b[tid] = sb3[tid];
      a.L3.mb[tid] = sb3[MC + tid];
      if (ADAM) a.L3.vb[tid] = sb3[2 * MC + tid];
    }
    if (tid < 4 && w + G * tid < N2) {
      const int n = w + G * tid;
      a.L2.b[n] = sb2[tid];
      a.L2.mb[n] = sb2[4 + tid];
      if (ADAM) a.L2.vb[n] = sb2[8 + tid];
    }
    if (fc1 && grp == 0 && tid < 16 && n0 + tid < N1) {
      const int n = n0 + tid;
      a.L1.b[n] = sb1[tid];
      a.L1.mb[n] = sb1[16 + tid];
      if (ADAM) a.L1.vb[n] = sb1[32 + tid];
    }
  }
}
#undef RES_IDX
#undef RES_MARK

int resident_lds_bytes(const ResArgs&) { return kResLds; }

static std::string check_shape(const ResArgs& a) {
  if (a.M < 1 || a.M > 16) return "rows per step 1..16";
  if (a.N1 < 1 || a.N1p > kSh1Max || a.N1p % 4) return "fc1 shard width <= 768";
  if (a.K1 % 4) return "fc1 input width % 4";
  if (a.N2 % 4 || a.N2 > kResRows2 * a.G || a.N2 > 1024) return "fc2 width % 4 and <= 4 G, <= 1024";
  if (a.C < 1 || a.C > kResMaxC || a.C4 % 4) return "classes <= 128";
  if (a.nfc1 > a.G || a.ngrp > kResGroups || a.nrb > kResMaxRB) return "fc1 tiles per workgroup";
  if (a.G > 256 || a.G < a.M) return "workgroups";
  if (a.ipc.T > 0 && ((int64_t)a.G * 64 * 2 > a.ipc.cap || a.ipc.T > kIpcMaxRanks))
    return "peer-mapped exchange region";
  return "";
}

bool resident_fits(const ResArgs& a, int device, std::string* why) {
  std::string s = check_shape(a);
  if (s.empty()) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, device) != hipSuccess) {
      s = "device properties";
    } else {
      // the instantiation that will be launched (Adam or SGD-momentum): their register counts differ
      const void* fn = a.o.kind == 2 ? reinterpret_cast<const void*>(&resident_epoch_kernel<true>)
                                     : reinterpret_cast<const void*>(&resident_epoch_kernel<false>);
      int nb = 0;
      const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kResThreads, kResLds);
      if (e != hipSuccess || nb < 1) s = "occupancy";
      else if ((int64_t)nb * pr.multiProcessorCount < a.G) s = "workgroups not co-resident";
    }
  }
  if (why) *why = s;
  return s.empty();
}

hipError_t resident_epoch_launch(const ResArgs& a, hipStream_t st) {
  if (!check_shape(a).empty()) return hipErrorInvalidValue;
  if (a.S <= 0) return hipSuccess;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&resident_epoch_kernel<true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kResLds);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&resident_epoch_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kResLds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipError_t e = hipMemsetAsync(a.cnt, 0, (size_t)kResCounters * kResShardStride * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  // cooperative: the runtime checks at launch time that all G workgroups fit at once (a
  // plain launch of a grid that does not fit would park workgroups behind ones that spin on
  // them); +15-19 us of host time per launch, once per client epoch (MI355X_MICROARCH.md)
  const void* fn = a.o.kind == 2 ? reinterpret_cast<const void*>(&resident_epoch_kernel<true>)
                                 : reinterpret_cast<const void*>(&resident_epoch_kernel<false>);
  ResArgs arg = a;
  if (!a.coop) {
    if (a.o.kind == 2)
      resident_epoch_kernel<true><<<a.G, kResThreads, kResLds, st>>>(a);
    else
      resident_epoch_kernel<false><<<a.G, kResThreads, kResLds, st>>>(a);
    return hipGetLastError();
  }
  void* params[] = {&arg};
  return hipLaunchCooperativeKernel(fn, dim3(a.G), dim3(kResThreads), params, (unsigned)kResLds, st);
}

}  // namespace sl
