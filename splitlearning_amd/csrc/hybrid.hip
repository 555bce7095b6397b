// Hybrid persistent server epoch: S steps of Bob's 3-layer tail in ONE launch for a wide
// shard (TP = 1 / 2 / 4 of model2_sisa), fc2 + head resident on-chip, fc1 streamed in-launch.
//
// Reference: bob.train_and_backward's inner loop (data_entities_vanilla_sisa.py:298-313), per
// cached batch `zero_grad; CE(model2_sisa(act), y).backward(); Adam.step()` (model2_sisa:
// fc1 5408 -> 5000, ReLU, dropout 0.5, fc2 5000 -> 1000, ReLU, dropout 0.5, fc3 1000 -> 100,
// models.py:46-63), for one tensor-parallel shard (fc1 column-, fc2 row-parallel, fc3
// replicated, as engine/tail.py).
//
// Why.  The launch-per-stage executor (engine.cpp) streams ALL of the shard's W / m / v
// through HBM every step (770 MB at TP = 1: 136 of the 170 us step) and pays six latency-
// bound launches (~35 us) around it; fc2's 120 MB of state plus two 20 MB reads of W2 (the
// forward and the data gradient) are part of that stream.  The register-resident epoch
// (resident.hip) removes the stream only where the whole shard fits on-chip (TP >= 7).  Here
// the part that fits stays: each of the G = 8 NC workgroups (one 8-wave workgroup per CU)
// holds one fc2 tile W2[r0 .. r0 + WR)[c0 .. c0 + WC) (<= 128 x 160: W in LDS, m / v in
// VGPRs), the head workgroups hold four fc3 columns, b2 and b3; fc1 streams.  Per step a
// workgroup moves only its ~27 fc1 tiles (16 x 256, W / m / v read and written once:
// 650 MB at TP = 1 instead of 770 + 40) plus hand-offs.
//
// Step i, workgroup w = (ta, tb) = (w / NC, w % NC):
//   F  wait until every fc1 row block overlapping fc2 column block tb has published its
//      look-ahead partials (counters R[rb]); h1[:, slice] = drop(relu(the partials summed in
//      workgroup order)) -> LDS (ta == 0 also -> H1 for the U phase's mask); the tile's fc2
//      partial FP[tb][r0 + n][m] = h1[m, slice] . W2[r0 + n, slice] (exact-fp32 MFMA) -> seam F
//   H  head w < N2 / 4 (fc2 rows 4w .. 4w + 3): P2 = the NC partials in order (tensor-
//      parallel: resident.hip's peer-mapped granule exchange, summed in rank order); h2 =
//      drop(relu(P2 + b2)); logit partials of these rows                      -> seam L
//   S  w < 4 M: quarter w % 4 of row w / 4's logits (partials in order, + b3) and its softmax
//      statistics {max, sum exp}                                                  -> seam D
//   H2 head: the softmax-CE from the logits and the quarters' statistics (loss by w = 0),
//      dz2 of its rows (dlogits . W3[:, rows], ReLU / dropout mask)              -> seam Z;
//      then the Adam steps of b3, its W3 columns and b2 (off the critical path)
//   B  the tile's dz1 partial DP[ta][m][c0 + j] = dz2[m, tile rows] . W2_i[tile rows, c0 + j]
//      (MFMA)                                                          -> counter P[tb];
//      then W2's Adam step in place (dW2 = dz2^T h1 of the tile, m / v in VGPRs)
//   U  fc1: dz1 of the workgroup's row blocks (the 8 partials in order, h1 > 0 mask, dropout
//      scale); b1's step (the row block's first workgroup); then its tile run: per 16 x 256
//      tile dW = dz1^T x_i, Adam on W / m / v, write-through stores, and the next batch's
//      look-ahead product x_{i+1} W1_{i+1}^T accumulated per row block (MFMA, the updated
//      tile staged through LDS as wgrad_group_kernel); the loads of the next tile are in
//      flight while a tile computes (first tile: issued before W2's update).  After the
//      run, each row block's partial (+ b1_{i+1} from its first workgroup) -> LA and one
//      arrival on R[rb]; step i + 1's F phases sum them (a last-arriving workgroup reducing
//      them first put a returning atomic, a cold read, a second publication and a second
//      counter on the critical path: 139.3 -> see docs/PERF.md round 5).
// A prologue pass (W1 read only) forms h1_0's partials the same way.  Arithmetic is fp32 (exact-fp32
// MFMA for the three products that use it); every sum runs in a fixed order, so a launch is
// deterministic and one launch of S steps is bitwise S one-step launches; the order differs
// from the launch-per-stage executor's, so results agree with it and with torch to fp32
// rounding (tests/test_hybrid_gpu.py).
//
// Hand-offs: write-through (sc1) payload stores, every wave drains (s_waitcnt vmcnt(0)), one
// agent-scope counter add per workgroup; consumers poll relaxed, then load with sc1 loads
// (MI355X_MICROARCH.md, the valid-forms table row 1).  Every wait is bounded (wall clock); a
// timeout raises err and every other wait gives up at once.  All G workgroups must be
// resident together: the host checks the launched instantiation's occupancy and launches
// cooperatively; nothing else may run on the device during the launch.
#include "hybrid.h"
#include "persist.h"

#include <string>

namespace sl {

namespace {

using namespace persist;

__device__ __forceinline__ unsigned* hy_cnt(const HyArgs& a, int i) { return a.cnt + i * kHyStride; }
__device__ __forceinline__ int hy_seam(int seam, int shard) { return seam * 8 + shard; }
__device__ __forceinline__ int hy_P(int b) { return kHySeams * 8 + b; }
__device__ __forceinline__ int hy_R(int rb) { return kHySeams * 8 + kHyMaxNC + rb; }

// bounded wait until *p >= tgt (one lane); false when it gave up
__device__ __forceinline__ bool hy_spin(const HyArgs& a, const unsigned* p, unsigned tgt) {
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

// every wave drains its write-through stores; the barrier orders the drains before the add
__device__ __forceinline__ void hy_arrive(const HyArgs& a, int idx) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(hy_cnt(a, idx), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the 8 shards of a seam (shard s receives shard_n[seam][s] arrivals per step)
// (s_sn: a.shard_n staged in LDS at the start, so the poll's target costs no global round trip)
__device__ __forceinline__ bool hy_seam_wait(const HyArgs& a, int seam, unsigned mult, int* s_ok, const int* s_sn) {
  int idx[8];
  unsigned tgt[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    idx[s] = hy_seam(seam, s);
    tgt[s] = mult * (unsigned)s_sn[seam * 8 + s];
  }
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < 8) {
      int id = idx[0];
      unsigned tg = tgt[0];
#pragma unroll
      for (int s = 1; s < 8; ++s)
        if (lane == s) {
          id = idx[s];
          tg = tgt[s];
        }
      if (tg > 0) ok = hy_spin(a, hy_cnt(a, id), tg);
    }
    ok = __all(ok);
    if (lane == 0) *s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return *s_ok != 0;
}

// fc1 state cache policy (buffer aux bits: 2 = non-temporal, 16 = write-through, 0 = plain).
// When the shard's state exceeds the 256 MB Infinity Cache (NTST, TP = 1: 325 MB with Adam),
// W is stored and loaded plain and m / v non-temporal, both ways: W's 108 MB then stay in the
// Infinity Cache from one step to the next while m / v stream past it without evicting it
// (TP = 1 144.7 us per step against 151.4 with every store non-temporal, 159.3 with every
// store write-through; W and m kept 149.2, W write-through 148.0;
// profiles/r4w_hybrid_per_array_cache_policy_ab.txt).  When it fits (TP = 2 / 4), every
// array write-through: 85.5 / 58.6 against 87.1 / 60.7 plain and 96.9 / 63.4 non-temporal.
// The same workgroup (same CU) reads a tile again next step.  On top, one workgroup in 4
// keeps its m tiles plain as well (27 MB more in the cache).  Round 4: one in 8 142.5-142.8 vs
// 144.8-145.0 without (one in 2 or 4: 143.3-143.8); on the round-6 kernel one in 4 is the better
// (two boxes, interleaved: 136.4-137.2 vs 137.4-138.1; a third neutral; all m plain 136.5-136.8
// vs 133.8-135.5 -- profiles/r6_hybrid/keep_m_ab.txt).
constexpr int kStW = 0, kStM = 2, kStV = 2;
constexpr int kLdW = 0, kLdM = 2, kLdV = 2;
constexpr int kKeepM = 3;
constexpr int kStFit = 16;

// fc2 column block of fc2 column (= fc1 shard row) float4 group n4: blocks [q0_b, q0_{b+1})
// with q0_b = floor(b Q4 / NC)
__device__ __forceinline__ int hy_colblk(int n4, int NC, int Q4) { return ((n4 + 1) * NC + Q4 - 1) / Q4 - 1; }

// LDS carve (bytes; offsets multiples of 16)
constexpr int PW2 = 4 * kHyMaxWC4 + 1;                 // W2 tile row pitch (floats)
constexpr int PH = 4 * kHyMaxWC4 + 4;                  // h1 slice row pitch (float4-aligned)
constexpr int PD = kHyMaxWR + 1;                       // dz2 slice row pitch
constexpr int OFF_W2 = 0;                              // W2 tile [kHyMaxWR][PW2]
constexpr int OFF_U = OFF_W2 + ((kHyMaxWR * PW2 * 4 + 15) & ~15);
// union, stream view
constexpr int U_SA = 0;                                // x_i tile [2][16][64] f32x4
constexpr int U_SW = U_SA + 2 * 16 * 64 * 16;          // updated W1 tile [2][16][65] f32x4
constexpr int kUStream = U_SW + 2 * 16 * 65 * 16;
// union, fc2 view
constexpr int U_SH1 = 0;                               // h1 slice [16][PH]
constexpr int U_SDZ2 = U_SH1 + 16 * PH * 4;            // dz2 slice [16][PD]
constexpr int U_RED = U_SDZ2 + ((16 * PD * 4 + 15) & ~15);   // [16][32] f32x4
constexpr int U_SDL = U_RED + 16 * 32 * 16;            // dlogits [16][kHyMaxC]
constexpr int U_SH2 = U_SDL + 16 * kHyMaxC * 4;        // h2 [16][4]
constexpr int U_SDZH = U_SH2 + 16 * 4 * 4;             // dz2 of the head rows [16][4]
constexpr int kUFc2 = U_SDZH + 16 * 4 * 4;
constexpr int kU = kUStream > kUFc2 ? kUStream : kUFc2;
constexpr int OFF_W3 = OFF_U + kU;                     // W3 columns {W, m, v}[4][kHyMaxC]
constexpr int OFF_B3 = OFF_W3 + 3 * 4 * kHyMaxC * 4;   // b3 {W, m, v}[kHyMaxC]
constexpr int OFF_B2 = OFF_B3 + 3 * kHyMaxC * 4;       // b2 {W, m, v}[4]
constexpr int OFF_B1 = OFF_B2 + 64;                    // b1 {W, m, v}[kHyRuns][16]
constexpr int OFF_DZ1 = OFF_B1 + kHyRuns * 3 * 16 * 4; // dz1 [kHyRuns][16 m][16 rows]
constexpr int OFF_OK = OFF_DZ1 + kHyRuns * 256 * 4;    // ints
// per-workgroup tile-table values the step loop needs, read from LDS instead of a global
// round trip on the critical path: the arrival counts of the F slice's row blocks [32] and
// this run's slots in its row blocks' partial lists [kHyRuns]
constexpr int OFF_TABC = OFF_OK + 64;
constexpr int kHyLds = OFF_TABC + (32 + kHyRuns + kHySeams * 8) * 4 + 4;
static_assert(kHyLds <= 160 * 1024, "LDS");
static_assert(kHyThreads / 64 * 10 * 256 >= kHyMaxWR * 4 * kHyMaxWC4, "10 W2 16 x 16 blocks per wave");

}  // namespace

// Per-lane indices from a laundered thread id at the top of every phase (as resident.hip:
// the compiler recomputes addresses where they are used instead of holding them across the
// step loop).  Thread (wave r of 8, lane): fc1 tile rows r and r + 8.
#define HY_IDX()                                                           \
  int tid_l_ = threadIdx.x;                                                \
  asm volatile("" : "+v"(tid_l_));                                         \
  const int tid = tid_l_, r = tid >> 6, lane = tid & 63, li = lane & 15, lq = lane >> 4; \
  (void)r; (void)lane; (void)li; (void)lq

// phase stamps (wall clock): workgroups 0 and G - 1 for the first trace_steps steps (trace), and
// every workgroup for steps tall_step .. tall_step + tall_n - 1 (tall [tall_n][G][16]: the
// critical-path table of scripts/hybrid_ab.py --trace)
#define HY_MARK(k)                                                                               \
  do {                                                                                           \
    if (threadIdx.x == 0) {                                                                      \
      if (a.trace != nullptr && i >= 0 && i < a.trace_steps && (w == 0 || w == G - 1))           \
        a.trace[((int64_t)(w == 0 ? 0 : 1) * a.trace_steps + i) * 16 + (k)] = (int64_t)wall_clock64(); \
      if (a.tall != nullptr && i >= a.tall_step && i < a.tall_step + a.tall_n)                   \
        a.tall[((int64_t)(i - a.tall_step) * G + w) * 16 + (k)] = (int64_t)wall_clock64();       \
    }                                                                                            \
  } while (0)

// NTST: fc1 state stores non-temporal (a shard whose streamed state is larger than the 256 MB
// Infinity Cache) or write-through (one that fits)
template <bool ADAM, bool NTST>
__global__ void __launch_bounds__(kHyThreads) hybrid_epoch_kernel(HyArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sw2 = reinterpret_cast<float*>(smem + OFF_W2);
  f32x4* sa = reinterpret_cast<f32x4*>(smem + OFF_U + U_SA);
  f32x4* sw = reinterpret_cast<f32x4*>(smem + OFF_U + U_SW);
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
  int* s_ok = reinterpret_cast<int*>(smem + OFF_OK);
  int* s_fns = reinterpret_cast<int*>(smem + OFF_TABC);        // [32]: ns of row block rlo + j
  int* s_slot = s_fns + 32;                                     // [kHyRuns]: w - first toucher
  int* s_sn = s_slot + kHyRuns;                                 // [kHySeams * 8]: a.shard_n
  constexpr int MC = kHyMaxC;
  const f32x4 zv = {0.f, 0.f, 0.f, 0.f};

  const int w = blockIdx.x;
  const int M = a.M, N1 = a.N1, K1 = a.K1, N2 = a.N2, C = a.C, C4 = a.C4, G = a.G, NC = a.NC;
  const int ncb = a.ncb;
  // fc2 tile (ta, tb): rows in groups of 4, columns in float4
  const int ta = w / NC, tb = w - (w / NC) * NC;
  const int Q2 = N2 >> 2, Q4 = N1 >> 2;
  const int r0 = 4 * (ta * Q2 / kHyNR), WR = 4 * ((ta + 1) * Q2 / kHyNR) - r0;
  const int q0 = tb * Q4 / NC, WC4 = (tb + 1) * Q4 / NC - q0;
  const int c0 = 4 * q0, WC = 4 * WC4;
  const bool head = w < a.HW;
  // fc1 tile run [t_begin, t_end), row blocks rbA .. rbA + nruns - 1
  const int t_begin = a.tab[w], t_end = a.tab[w + 1];
  const int nt = t_end - t_begin;
  const int rbA = nt > 0 ? t_begin / ncb : 0;
  const int nruns = nt > 0 ? (t_end - 1) / ncb - rbA + 1 : 0;
  // every hand-off buffer through one resource (offsets in bytes: base + element * 4)
  const __amdgpu_buffer_rsrc_t rHB = rs_of(a.HB);
  const int bLA = 4 * a.oLA, bH1 = 4 * a.oH1, bFP = 4 * a.oFP, bLP = 4 * a.oLP, bDL = 4 * a.oDL, bDZ = 4 * a.oDZ,
            bDP = 4 * a.oDP, bZP = 4 * a.oZP;
  const __amdgpu_buffer_rsrc_t rW1 = rs_of(a.L1.W), rM1 = rs_of(a.L1.m), rV1 = rs_of(a.L1.v ? a.L1.v : a.L1.m);

  // ---- load the resident state: the W2 tile (LDS), its m / v (VGPRs), head columns, biases
  f32x4 m2[10], v2[10];
  {
    HY_IDX();
    for (int e = tid; e < kHyMaxWR * PW2; e += kHyThreads) sw2[e] = 0.f;
    __syncthreads();
    for (int e = tid; e < WR * WC4; e += kHyThreads) {
      const int n = e / WC4, q = e - n * WC4;
      const f32x4 wv = *reinterpret_cast<const f32x4*>(a.L2.W + (int64_t)(r0 + n) * N1 + c0 + 4 * q);
#pragma unroll
      for (int k = 0; k < 4; ++k) sw2[n * PW2 + 4 * q + k] = wv[k];
    }
    // m / v of the tile in the 16 x 16 MFMA accumulator layout of W2's update: block b = r + 8 u
    // (rows 16 (b / 10) .., columns 16 (b % 10) ..), lane (li, lq) holds rows 4 lq + j, column li
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int b = r + 8 * u, bn = b / 10, bk = b - (b / 10) * 10;
      m2[u] = v2[u] = zv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * bn + 4 * lq + j, k = 16 * bk + li;
        if (n < WR && k < WC) {
          const int64_t off = (int64_t)(r0 + n) * N1 + c0 + k;
          m2[u][j] = a.L2.m[off];
          if (ADAM) v2[u][j] = a.L2.v[off];
        }
      }
    }
    if (head && tid < 4 * MC) {
      const int ii = tid / MC, c = tid - ii * MC;
      const int n = 4 * w + ii;
      const bool ok = c < C;
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
    if (head && tid < 4) {
      const int n = 4 * w + tid;
      sb2[tid] = a.L2.b[n];
      sb2[4 + tid] = a.L2.mb[n];
      sb2[8 + tid] = ADAM ? a.L2.vb[n] : 0.f;
    }
    if (tid < 32) {
      const int rb = (c0 >> 4) + tid;
      s_fns[tid] = rb <= ((c0 + WC - 1) >> 4) && rb < a.nrb ? a.tab[a.G + 1 + a.nrb + rb] : 0;
    }
    if (tid < kHyRuns) s_slot[tid] = tid < nruns ? w - a.tab[a.G + 1 + rbA + tid] : -1;
    if (tid < kHySeams * 8) s_sn[tid] = a.shard_n[tid];
    if (tid < 16 * kHyRuns) {
      const int k = tid >> 4, j = tid & 15;
      const int rb = rbA + k, n = 16 * rb + j;
      const bool own = k < nruns && a.tab[a.G + 1 + rb] == w && n < N1;
      sb1[(k * 3 + 0) * 16 + j] = own ? a.L1.b[n] : 0.f;
      sb1[(k * 3 + 1) * 16 + j] = own ? a.L1.mb[n] : 0.f;
      sb1[(k * 3 + 2) * 16 + j] = (own && ADAM) ? a.L1.vb[n] : 0.f;
    }
  }

  // ---------------------------------------------------------------- fc1 tile stream
  // state of tile t (rows n0 + r + 8h, float4 column kb + 4 lane) into p / m / v
  // over the cache (NTST): the workgroups w % (kKeepM + 1) == 0 keep their m tiles plain too
  const bool mkeep = NTST && (w & kKeepM) == 0;
  auto load_state = [&](int t, f32x4 (&p)[2], f32x4 (&mm)[2], f32x4 (&vv)[2], bool upd) {
    HY_IDX();
    const int rb = t / ncb, cb = t - (t / ncb) * ncb;
    const int k = cb * 256 + 4 * lane;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = 16 * rb + r + 8 * h;
      const bool act = n < N1 && k < K1;
      const int boff = (n * K1 + k) * 4;
      p[h] = act ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rW1, boff, 0, NTST ? kLdW : 0)) : zv;
      if (upd) {
        mm[h] = act ? (mkeep ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rM1, boff, 0, 0))
                             : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rM1, boff, 0, NTST ? kLdM : 0)))
                    : zv;
        vv[h] = (act && ADAM) ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rV1, boff, 0, NTST ? kLdV : 0)) : zv;
      }
    }
  };
  // x rows r, r + 8 of tile t's 256 columns (dW operand, staged in LDS)
  const __amdgpu_buffer_rsrc_t rX = rs_of(a.X);
  auto load_xa = [&](int row0, int t, f32x4 (&xa)[2]) {
    HY_IDX();
    const int cb = t - (t / ncb) * ncb;
    const int k = cb * 256 + 4 * lane;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = r + 8 * h;
      xa[h] = (m < M && k < K1)
                  ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rX, ((row0 + m) * K1 + k) * 4, 0, 0))
                  : zv;
    }
  };
  // next batch's rows in MFMA A layout: lane (li, lq) of wave r, column group r + 8 h
  auto load_xv = [&](int row0, int t, f32x4 (&xv)[2]) {
    HY_IDX();
    const int cb = t - (t / ncb) * ncb;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = cb * 256 + 16 * (r + 8 * h) + 4 * lq;
      xv[h] = (li < M && k < K1)
                  ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rX, ((row0 + li) * K1 + k) * 4, 0, 0))
                  : zv;
    }
  };

  // fc1 state stores: the policy above (kSt*, kStFit)
  auto sst4 = [&](auto sp_c, __amdgpu_buffer_rsrc_t rs, int boff, f32x4 v) {
    constexpr int SP = NTST ? decltype(sp_c)::value : kStFit;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(res_i32x4, v), rs, boff, 0, SP);
  };
  using StW = std::integral_constant<int, kStW>;
  using StM = std::integral_constant<int, kStM>;
  using StV = std::integral_constant<int, kStV>;

  // One pass over this workgroup's tile run.  UPD: dW = dz1^T x_t and the optimizer step
  // (false: the prologue's read-only pass); LOOK: the look-ahead product with xn, per wave an
  // MFMA accumulator per row block, stored to ZP when the run leaves the row block.  sp / sm /
  // sv [0] hold tile t_begin's state, already issued.
  f32x4 sp[2][2], sm[2][2], sv[2][2];
  f32x4 zlast = zv;
  auto zp_store = [&](int k, f32x4 z) {
    HY_IDX();
    hst4(rHB, bZP + (((w * kHyRuns + k) * 8 + r) * 64 + lane) * 16, z);
  };
  auto stream = [&](auto upd_c, auto look_c, int xt, int xn, float ss, float ib) {
    constexpr bool UPD = decltype(upd_c)::value, LOOK = decltype(look_c)::value;
    if (nt <= 0) return;
    f32x4 xa[2], xv[2];
    if (UPD) {
      load_xa(xt, t_begin, xa);
      HY_IDX();
      sa[r * 64 + lane] = xa[0];
      sa[(r + 8) * 64 + lane] = xa[1];
    }
    __syncthreads();
    f32x4 z = zv;
    int kz = 0;   // run index of the row block z accumulates
    auto tile = [&](auto cur_c, int j) {
      constexpr int cur = decltype(cur_c)::value, nb = cur ^ 1;
      const int t = t_begin + j;
      const int rb = t / ncb, cb = t - (t / ncb) * ncb;
      const int kr = rb - rbA;
      if (LOOK && kr != kz) {   // uniform: the run entered its next row block
        zp_store(kz, z);
        z = zv;
        kz = kr;
      }
      // loads first, in the order they are consumed (a wave's loads complete in order): the next
      // tile's x operand (staged at the end of this tile), this tile's look-ahead operand, then
      // the next tile's state (consumed one tile later)
      if (UPD && j + 1 < nt) load_xa(xt, t + 1, xa);
      if (LOOK) load_xv(xn, t, xv);
      if (j + 1 < nt) load_state(t + 1, sp[nb], sm[nb], sv[nb], UPD);
      HY_IDX();
      const int n1 = 16 * rb + r;
      const int k = cb * 256 + 4 * lane;
      const bool kin = k < K1;
      if (UPD) {
        const float* dz = sdz1 + kr * 256;
        // (unroll 4: fully unrolled, the 16 x loads and 32 dz1 scalars were all hoisted, ~100
        // VGPRs, which spilled the fc2 state)
        f32x4 g0 = zv, g1 = zv;
#pragma unroll 4
        for (int m = 0; m < 16; ++m) {
          const f32x4 xm = sa[cur * 1024 + m * 64 + lane];
          g0 += dz[m * 16 + r] * xm;
          g1 += dz[m * 16 + r + 8] * xm;
        }
        if (kin && n1 < N1) {
          res_update4<ADAM>(a.o, ss, ib, sp[cur][0], g0, sm[cur][0], sv[cur][0]);
          const int boff = (n1 * K1 + k) * 4;
          sst4(StW{}, rW1, boff, sp[cur][0]);
          if (mkeep) sst4(std::integral_constant<int, 0>{}, rM1, boff, sm[cur][0]);
          else sst4(StM{}, rM1, boff, sm[cur][0]);
          if (ADAM) sst4(StV{}, rV1, boff, sv[cur][0]);
        }
        if (kin && n1 + 8 < N1) {
          res_update4<ADAM>(a.o, ss, ib, sp[cur][1], g1, sm[cur][1], sv[cur][1]);
          const int boff = ((n1 + 8) * K1 + k) * 4;
          sst4(StW{}, rW1, boff, sp[cur][1]);
          if (mkeep) sst4(std::integral_constant<int, 0>{}, rM1, boff, sm[cur][1]);
          else sst4(StM{}, rM1, boff, sm[cur][1]);
          if (ADAM) sst4(StV{}, rV1, boff, sv[cur][1]);
        }
        if (j + 1 < nt) {
          sa[nb * 1024 + r * 64 + lane] = xa[0];
          sa[nb * 1024 + (r + 8) * 64 + lane] = xa[1];
        }
      }
      if (LOOK) {
        sw[cur * 1040 + r * 65 + lane] = (kin && n1 < N1) ? sp[cur][0] : zv;
        sw[cur * 1040 + (r + 8) * 65 + lane] = (kin && n1 + 8 < N1) ? sp[cur][1] : zv;
      }
      __syncthreads();
      if (LOOK) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 wv4 = sw[cur * 1040 + li * 65 + 4 * (r + 8 * h) + lq];
#pragma unroll
          for (int c = 0; c < 4; ++c) z = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[h][c], wv4[c], z, 0, 0, 0);
        }
      }
    };
    int j = 0;
    for (; j + 1 < nt; j += 2) {
      tile(std::integral_constant<int, 0>{}, j);
      tile(std::integral_constant<int, 1>{}, j + 1);
    }
    if (j < nt) tile(std::integral_constant<int, 0>{}, j);
    zlast = z;   // the last row block's accumulators go to flush through LDS
  };

  // Publish the run's look-ahead partials for step `so` (parity so & 1): each row block's
  // partial (the 8 waves' MFMA accumulators from ZP, in wave order, + b1 by its first
  // workgroup) -> LA, then one arrival per row block on R[].  The consumers (step so's F) sum a
  // row block's partials in workgroup order and apply its epilogue themselves: no last-arriver
  // round trip, no second publication on the step's critical path.
  auto flush = [&](int so) {
    const int par = so & 1;
    {
      // the last row block's per-wave accumulators through LDS (the stream's buffers are free
      // once every wave passed this barrier); earlier row blocks' from ZP
      HY_IDX();
      __syncthreads();
      sa[r * 64 + lane] = zlast;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    {
      const int i = so - 1;   // trace: the drain of the run's last stores ends (stamp 15)
      HY_MARK(15);
    }
    {
      HY_IDX();
      // (row nn, rows m = 4 mg ..): the waves' accumulators are already in that layout
      for (int e = tid; e < nruns * 64; e += kHyThreads) {
        const int k = e >> 6, nn = (e >> 2) & 15, mg = e & 3;
        const int rb = rbA + k, slot = s_slot[k], n = 16 * rb + nn;
        f32x4 parts[8];
        if (k == nruns - 1) {
#pragma unroll
          for (int ww = 0; ww < 8; ++ww) parts[ww] = sa[ww * 64 + 16 * mg + nn];
        } else {
#pragma unroll
          for (int ww = 0; ww < 8; ++ww) parts[ww] = hld4(rHB, bZP + (((w * kHyRuns + k) * 8 + ww) * 64 + 16 * mg + nn) * 16);
        }
        f32x4 v = parts[0];
#pragma unroll
        for (int ww = 1; ww < 8; ++ww) v += parts[ww];
        if (slot == 0) v += sb1[(k * 3) * 16 + nn];
        if (n < N1) hst4(rHB, bLA + (((par * a.nrb + rb) * kHySlots + slot) * 256 + nn * 16 + 4 * mg) * 4, v);
      }
    }
    // every wave drained its LA stores; then one lane per run row block arrives
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < (unsigned)nruns)
      __hip_atomic_fetch_add(hy_cnt(a, hy_R(rbA + threadIdx.x)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // ---- prologue: h1_0 = drop(relu(x_0 W1_0^T + b1)) by a read-only pass over the run
  if (nt > 0) load_state(t_begin, sp[0], sm[0], sv[0], false);
  stream(std::false_type{}, std::true_type{}, 0, 0, 0.f, 0.f);
  flush(0);

  for (int i = 0; i < a.S; ++i) {
    const int par = i & 1;
    const bool more = i + 1 < a.S;
    const uint32_t sd2 = a.seeds[4 * i + 2], sd3 = a.seeds[4 * i + 3];
    const SlOpt o = a.o;
    float ss = ADAM ? a.adam[4 * i] : 0.f, ib = ADAM ? a.adam[4 * i + 1] : 0.f;
    asm volatile("" : "+v"(ss), "+v"(ib));

    // ================= F: h1 slice, the tile's fc2 partial
    HY_MARK(0);
    // the look-ahead partials of every fc1 row block overlapping this column block
    // [c0, c0 + WC) published (R[rb] counts each run's arrival: (i + 1) ns[rb] by now; lane l of
    // wave 0 polls row block rlo + l)
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      const int rlo = c0 >> 4, rhi = (c0 + WC - 1) >> 4;
      bool ok = true;
      if (rlo + lane <= rhi) {
        const int rb = rlo + lane;
        // fault injection (tests): at step fault_step this wait cannot be met, times out (err 2)
        // and every other wait gives up, as a hand-off that never arrives would make them
        const unsigned tg = i == a.fault_step ? 0xffffffffu : (unsigned)(i + 1) * (unsigned)s_fns[lane];
        ok = hy_spin(a, hy_cnt(a, hy_R(rb)), tg);
      }
      ok = __all(ok);
      if (lane == 0) *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (*s_ok == 0) break;
    HY_MARK(1);
    {
      // h1 of the slice from the partials (in workgroup order; slot 0 carries b1), ReLU and
      // step i's dropout, rows m >= M zero, columns >= WC zero; the ta == 0 workgroup also
      // publishes it to H1 ([N1][16]: the U phase's ReLU mask)
      HY_IDX();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = tid + u * kHyThreads;
        const int kc = e >> 2, mg = e & 3;
        if (kc < 4 * kHyMaxWC4) {
          f32x4 v = zv;
          if (kc < WC) {
            const int n = c0 + kc, rb = n >> 4, nn = n & 15;
            const int ns = s_fns[rb - (c0 >> 4)];
            f32x4 parts[kHySlots];
#pragma unroll
            for (int sl = 0; sl < kHySlots; ++sl)
              parts[sl] = sl < ns ? hld4(rHB, bLA + (((par * a.nrb + rb) * kHySlots + sl) * 256 + nn * 16 + 4 * mg) * 4) : zv;
            v = parts[0];
#pragma unroll
            for (int sl = 1; sl < kHySlots; ++sl) v += parts[sl];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int m = 4 * mg + j;
              v[j] = m < M ? drop_relu(v[j], a.seeds[4 * i], a.seeds[4 * i + 1], m, a.col_off1 + n, a.thr1, a.dsc1) : 0.f;
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
      HY_IDX();
      if (16 * r < WR) {
        f32x4 acc0 = zv, acc1 = zv;
        const float* pa = sh1 + li * PH + lq;
        const float* pb = sw2 + (16 * r + li) * PW2 + lq;
#pragma unroll
        for (int kk = 0; kk < kHyMaxWC4; kk += 2) {
          if (kk < WC4) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * kk], pb[4 * kk], acc0, 0, 0, 0);
          if (kk + 1 < WC4) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * kk + 4], pb[4 * kk + 4], acc1, 0, 0, 0);
        }
        const f32x4 acc = acc0 + acc1;
        const int n = 16 * r + li;
        // FP is [NC][N2][16]: the lane's four rows m = 4 lq .. as one 16-B store
        if (n < WR) hst4(rHB, bFP + (((par * NC + tb) * N2 + r0 + n) * 16 + 4 * lq) * 4, acc);
      }
    }
    hy_arrive(a, hy_seam(0, w & 7));
    HY_MARK(2);

    // ================= H: P2 of the head rows, h2, logit partials
    if (head) {
      if (!hy_seam_wait(a, 0, (unsigned)(i + 1), s_ok, s_sn)) break;
      HY_MARK(3);
      {
        // partial cq of fc2 row 4 w + ii, rows m = 4 mg .. (FP is [NC][N2][16])
        HY_IDX();
        const int cq = tid >> 4, ii = (tid >> 2) & 3, mg = tid & 3;
        red[tid] = cq < NC ? hld4(rHB, bFP + (((par * NC + cq) * N2 + 4 * w + ii) * 16 + 4 * mg) * 4) : zv;
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        HY_IDX();
        const int m = tid >> 2, ii = tid & 3;
        // the NC partials in order (partials >= NC are zero)
        float pv = red[ii * 4 + (m >> 2)][m & 3];
#pragma unroll
        for (int cq = 1; cq < kHyMaxNC; ++cq) pv += red[cq * 16 + ii * 4 + (m >> 2)][m & 3];
        if (a.ipc.T > 0) {
          // tensor-parallel fc2 (row-parallel): this workgroup's 16 x 4 product block to every
          // rank as 8-byte granules {generation, value}, summed in rank order on every rank
          // (resident.hip's exchange; region reuse is ordered by the exchange itself)
          const uint32_t gen = a.ipc.gen + (uint32_t)i;
          const int ipar = (int)(gen & 1u), T = a.ipc.T, me = a.ipc.me;
          const int64_t half = a.ipc.cap >> 1;
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
        const int n = 4 * w + ii;
        sh2[m * 4 + ii] = m < M ? drop_relu(pv + sb2[ii], sd2, sd3, m, n, a.thr2, a.dsc2) : 0.f;
      }
      __syncthreads();
      if (a.ipc.T > 0 && *s_ok == 0) break;
      {
        HY_IDX();
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
      hy_arrive(a, hy_seam(1, w & 7));
      HY_MARK(4);
    }

    // ================= S: row m's logits, softmax-CE, dlogits (workgroups m < M)
    if (w < M) {
      if (!hy_seam_wait(a, 1, (unsigned)(i + 1), s_ok, s_sn)) break;
      HY_MARK(5);
      const int m = w;
      const int nc4 = C4 >> 2;
      constexpr int NG = kHyThreads / 32;                 // 16 partial-sum groups
      {
        HY_IDX();
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
        HY_IDX();
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
        if (act) hst4(rHB, bDL + ((par * 16 + m) * C4 + 4 * c4) * 4, d);
        if (tid == 0) a.loss[(int64_t)i * M + m] = ign ? 0.f : mx + logf(se) - zl;
      }
      hy_arrive(a, hy_seam(2, w & 7));
      HY_MARK(6);
    }

    // ================= H2: dz2 of the head rows; b3 / W3 / b2 steps
    if (head) {
      if (!hy_seam_wait(a, 2, (unsigned)(i + 1), s_ok, s_sn)) break;
      HY_MARK(7);
      {
        HY_IDX();
        for (int e = tid; e < 16 * (MC / 4); e += kHyThreads) {
          const int m = e / (MC / 4), c = 4 * (e - m * (MC / 4));
          *reinterpret_cast<f32x4*>(sdl + m * MC + c) = (m < M && c < C4) ? hld4(rHB, bDL + ((par * 16 + m) * C4 + c) * 4) : zv;
        }
      }
      __syncthreads();
      {
        HY_IDX();
        // dh2[m][ii] = sum_c dlog[m][c] W3[c][4 w + ii] (old W3): 16 lanes per (m, ii)
#pragma unroll
        for (int oi0 = 0; oi0 < 64; oi0 += kHyThreads / 16) {
          const int oi = oi0 + (tid >> 4), part = tid & 15;
          const int m = oi >> 2, ii = oi & 3;
          float s = 0.f;
#pragma unroll
          for (int cc = 0; cc < MC; cc += 16) s = fmaf(sdl[m * MC + cc + part], sW3[ii * MC + cc + part], s);
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
      hy_arrive(a, hy_seam(3, w & 7));
      HY_MARK(8);
      {
        HY_IDX();
        if (tid < C) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdl[m * MC + tid];   // rows >= M are zero
          res_update<ADAM>(o, ss, ib, sb3[tid], g, sb3[MC + tid], sb3[2 * MC + tid]);
        }
        for (int e = tid; e < 4 * MC; e += kHyThreads) {
          const int ii = e / MC, c = e - ii * MC;
          if (c < C) {
            float g = 0.f;
#pragma unroll
            for (int m = 0; m < 16; ++m) g = fmaf(sdl[m * MC + c], sh2[m * 4 + ii], g);
            res_update<ADAM>(o, ss, ib, sW3[ii * MC + c], g, sW3[(4 + ii) * MC + c], sW3[(8 + ii) * MC + c]);
          }
        }
        if (tid < 4) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdzh[m * 4 + tid];
          res_update<ADAM>(o, ss, ib, sb2[tid], g, sb2[4 + tid], sb2[8 + tid]);
        }
      }
    }

    // ================= B: the tile's dz1 partial, then W2's step
    if (!hy_seam_wait(a, 3, (unsigned)(i + 1), s_ok, s_sn)) break;
    HY_MARK(9);
    {
      HY_IDX();
      const int m = tid >> 5, k4 = tid & 31;   // 16 rows x 32 float4 (WR <= 128)
      const f32x4 v = (m < M && 4 * k4 < WR) ? hld4(rHB, bDZ + ((par * 16 + m) * N2 + r0 + 4 * k4) * 4) : zv;
#pragma unroll
      for (int k = 0; k < 4; ++k) sdz2[m * PD + 4 * k4 + k] = v[k];
    }
    __syncthreads();
    {
      // wave r: column tiles r and r + 8 of the slice (16 columns each); K = the tile's rows
      HY_IDX();
      const int jt0 = r, jt1 = r + 8;
      const bool two = 16 * jt1 < WC;
      if (16 * jt0 < WC) {
        f32x4 a0 = zv, a1 = zv, b0 = zv, b1 = zv;
        const float* pa = sdz2 + li * PD + lq;
        const float* pb0 = sw2 + lq * PW2 + 16 * jt0 + li;
        const float* pb1 = sw2 + lq * PW2 + 16 * (two ? jt1 : jt0) + li;
#pragma unroll
        for (int kk = 0; kk < kHyMaxWR / 4; kk += 2) {
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
          // DP is [8][N1][16]: the lane's four rows m = 4 lq .. as one 16-B store
          if (j < WC) hst4(rHB, bDP + (((par * kHyNR + ta) * N1 + c0 + j) * 16 + 4 * lq) * 4, acc);
        }
      }
    }
    hy_arrive(a, hy_P(tb));
    HY_MARK(10);
    // the first fc1 tile's state in flight under W2's update and the dz1 wait
    if (nt > 0) load_state(t_begin, sp[0], sm[0], sv[0], true);
    {
      // dW2 of the tile = dz2[:, rows]^T h1[:, slice] on exact-fp32 MFMA (K = the 16 batch rows),
      // each wave 10 blocks of 16 x 16, the moments already in the accumulator layout; W2 in LDS
      // updated in place (a VALU form with the dz2 / h1 operands re-read from LDS per element
      // took 9.8 us of the critical path)
      HY_IDX();
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
          res_update4<ADAM>(o, ss, ib, p, g, m2[u], v2[u]);
#pragma unroll
          for (int j = 0; j < 4; ++j) sw2[(16 * bn + 4 * lq + j) * PW2 + 16 * bk + li] = p[j];
        }
      }
    }
    HY_MARK(11);

    // ================= U: fc1 dz1, b1's step, the tile stream, the look-ahead publication
    {
      // the dz1 partials of every fc2 column block covering this run's row blocks (a contiguous
      // range; lane l of wave 0 polls block blo + l)
      if (nruns > 0 && threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const int blo = hy_colblk((16 * rbA) >> 2, NC, Q4);
        const int bhi = hy_colblk((min(16 * (rbA + nruns), N1) - 1) >> 2, NC, Q4);
        bool ok = true;
        if (blo + lane <= bhi) ok = hy_spin(a, hy_cnt(a, hy_P(blo + lane)), (unsigned)(i + 1) * kHyNR);
        ok = __all(ok);
        if (lane == 0) *s_ok = ok ? 1 : 0;
      }
      __syncthreads();
      if (nruns > 0 && *s_ok == 0) break;
    }
    HY_MARK(12);
    {
      HY_IDX();
      // (row nn, rows m = 4 mg ..): DP is [8][N1][16], H1 [N1][16]
      for (int e = tid; e < kHyRuns * 64; e += kHyThreads) {
        const int k = e >> 6, nn = (e >> 2) & 15, mg = e & 3;
        const int n = 16 * (rbA + k) + nn;
        f32x4 v = zv;
        if (k < nruns && n < N1) {
          f32x4 parts[kHyNR];
#pragma unroll
          for (int b = 0; b < kHyNR; ++b) parts[b] = hld4(rHB, bDP + (((par * kHyNR + b) * N1 + n) * 16 + 4 * mg) * 4);
          const f32x4 h = hld4(rHB, bH1 + ((par * N1 + n) * 16 + 4 * mg) * 4);
          v = parts[0];
#pragma unroll
          for (int b = 1; b < kHyNR; ++b) v += parts[b];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (4 * mg + j < M && h[j] > 0.f) ? v[j] * a.dsc1 : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) sdz1[k * 256 + (4 * mg + j) * 16 + nn] = v[j];
      }
    }
    __syncthreads();
    {
      HY_IDX();
      if (tid < 16 * nruns) {
        const int k = tid >> 4, jj = tid & 15;
        const int rb = rbA + k;
        if (s_slot[k] == 0 && 16 * rb + jj < N1) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < 16; ++m) g += sdz1[k * 256 + m * 16 + jj];
          res_update<ADAM>(o, ss, ib, sb1[(k * 3) * 16 + jj], g, sb1[(k * 3 + 1) * 16 + jj], sb1[(k * 3 + 2) * 16 + jj]);
        }
      }
    }
    const int xt = i * M, xn = (i + 1) * M;   // first rows of this / the next batch in X
    if (more) {
      stream(std::true_type{}, std::true_type{}, xt, xn, ss, ib);
      HY_MARK(13);
      flush(i + 1);
    } else {
      stream(std::true_type{}, std::false_type{}, xt, xn, ss, ib);
    }
    HY_MARK(14);
  }

  // ---- write the resident state back
  __syncthreads();
  {
    HY_IDX();
    for (int e = tid; e < WR * WC4; e += kHyThreads) {
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
        if (n < WR && k < WC) {
          const int64_t off = (int64_t)(r0 + n) * N1 + c0 + k;
          a.L2.m[off] = m2[u][j];
          if (ADAM) a.L2.v[off] = v2[u][j];
        }
      }
    }
    if (head && tid < 4 * MC) {
      const int ii = tid / MC, c = tid - ii * MC;
      if (c < C) {
        const int64_t off = (int64_t)c * N2 + 4 * w + ii;
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
    if (head && tid < 4) {
      const int n = 4 * w + tid;
      a.L2.b[n] = sb2[tid];
      a.L2.mb[n] = sb2[4 + tid];
      if (ADAM) a.L2.vb[n] = sb2[8 + tid];
    }
    if (tid < 16 * nruns) {
      const int k = tid >> 4, j = tid & 15;
      const int rb = rbA + k, n = 16 * rb + j;
      if (a.tab[a.G + 1 + rb] == w && n < N1) {
        a.L1.b[n] = sb1[(k * 3 + 0) * 16 + j];
        a.L1.mb[n] = sb1[(k * 3 + 1) * 16 + j];
        if (ADAM) a.L1.vb[n] = sb1[(k * 3 + 2) * 16 + j];
      }
    }
  }
}
#undef HY_IDX
#undef HY_MARK

int hybrid_lds_bytes() { return kHyLds; }

// the instantiation a launch uses: Adam / SGD-momentum, non-temporal or write-through state stores
static const void* hybrid_fn(const HyArgs& a) {
  if (a.o.kind == 2)
    return a.ntst ? reinterpret_cast<const void*>(&hybrid_epoch_kernel<true, true>)
                  : reinterpret_cast<const void*>(&hybrid_epoch_kernel<true, false>);
  return a.ntst ? reinterpret_cast<const void*>(&hybrid_epoch_kernel<false, true>)
                : reinterpret_cast<const void*>(&hybrid_epoch_kernel<false, false>);
}

std::string hybrid_check(const HyArgs& a) {
  if (a.M < 1 || a.M > 16) return "rows per step 1..16";
  if (a.G < 8 || a.G % kHyNR || a.NC != a.G / kHyNR || a.NC > kHyMaxNC) return "workgroups (8 x column blocks)";
  if (a.N1 < 4 || a.N1 % 4) return "fc1 shard width % 4";
  if ((a.N1 / 4 + a.NC - 1) / a.NC > kHyMaxWC4) return "fc1 shard too wide for the fc2 tiles";
  if (a.N1 > 16 * kHyMaxRB || a.nrb != (a.N1 + 15) / 16) return "fc1 row blocks";
  if (a.K1 % 4 || a.K1 < 4 || a.ncb != (a.K1 + 255) / 256) return "fc1 input width % 4";
  if ((int64_t)a.N1 * a.K1 * 4 > 2147483647LL) return "fc1 larger than 2 GB (32-bit buffer offsets)";
  if ((int64_t)a.S * a.M * a.K1 * 4 > 2147483647LL) return "epoch inputs larger than 2 GB (32-bit buffer offsets)";
  if (a.N2 < 4 || a.N2 % 4 || a.N2 > 4 * a.G || 4 * ((a.N2 / 4 + kHyNR - 1) / kHyNR) > kHyMaxWR || a.HW != a.N2 / 4)
    return "fc2 width % 4, <= 1024";
  if (a.C < 1 || a.C > kHyMaxC || a.C4 != ((a.C + 3) & ~3)) return "classes <= 128";
  if (a.G < a.M) return "workgroups < rows";
  if (a.ipc.T > 0 && ((int64_t)a.HW * 64 * 2 > a.ipc.cap || a.ipc.T > kIpcMaxRanks)) return "peer-mapped exchange region";
  return "";
}

bool hybrid_fits(const HyArgs& a, int device, std::string* why) {
  std::string s = hybrid_check(a);
  if (s.empty()) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, device) != hipSuccess) {
      s = "device properties";
    } else {
      const void* fn = hybrid_fn(a);
      int nb = 0;
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kHyLds);
      if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kHyThreads, kHyLds);
      if (e != hipSuccess || nb < 1) s = "occupancy";
      else if ((int64_t)nb * pr.multiProcessorCount < a.G) s = "workgroups not co-resident";
    }
  }
  if (why) *why = s;
  return s.empty();
}

hipError_t hybrid_epoch_launch(const HyArgs& a, hipStream_t st) {
  if (!hybrid_check(a).empty()) return hipErrorInvalidValue;
  if (a.S <= 0) return hipSuccess;
  const void* fn = hybrid_fn(a);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kHyLds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.cnt, 0, (size_t)kHyCounters * kHyStride * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  HyArgs arg = a;
  if (!a.coop) {
    void* params[] = {&arg};
    return hipLaunchKernel(fn, dim3(a.G), dim3(kHyThreads), params, (size_t)kHyLds, st);
  }
  void* params[] = {&arg};
  return hipLaunchCooperativeKernel(fn, dim3(a.G), dim3(kHyThreads), params, (unsigned)kHyLds, st);
}

}  // namespace sl
