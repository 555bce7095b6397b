// Hybrid persistent server epoch (csrc/hybrid.hip): S Adam/SGD steps of Bob's 3-layer tail in
// ONE launch for a WIDE shard (TP = 1 / 2 / 4 of model2_sisa: fc1 5000 / 2500 / 1250 x 5408),
// whose state does not fit on-chip.  fc2 (W in LDS, m / v in VGPRs), fc3 and the biases stay
// on-chip for the whole epoch; fc1's W / m / v stream through the launch once per step, each
// workgroup walking a fixed run of 16 x 256 tiles with the next tile's loads in flight.
#pragma once
#include "common.h"
#include "ipc_ar.h"
#include "resident.h"

namespace sl {

constexpr int kHyThreads = 512;     // one 8-wave workgroup per CU (256 VGPRs per wave)
constexpr int kHyNR = 8;            // fc2 row blocks (tile rows 4 ceil(N2 / 32) <= 128)
constexpr int kHyMaxNC = 32;        // fc2 column blocks (G = 8 NC)
constexpr int kHyMaxWR = 128;       // fc2 tile rows
constexpr int kHyMaxWC4 = 40;       // fc2 tile columns / 4 (160)
constexpr int kHyMaxC = 128;        // classes
constexpr int kHyRuns = 3;          // fc1 row blocks one workgroup's tile run may touch
constexpr int kHySlots = 8;         // workgroups whose runs may touch one fc1 row block
constexpr int kHyMaxRB = 320;       // fc1 row blocks of 16 rows (N1 <= 5120)
constexpr int kHyStride = 32;       // counter words 128 B apart
constexpr int kHySeams = 4;         // F: fc2 partials, L: logit partials, D: dlogits, Z: dz2
// counter words: the seams' 8 shards each, then P[NC] (dz1 partials per fc2 column block),
// R[nrb] (look-ahead partials per fc1 row block)
constexpr int kHyCounters = kHySeams * 8 + kHyMaxNC + kHyMaxRB;

struct HyArgs {
  ResLayer L1, L2, L3;
  int N1, K1, N2, C;      // shard fc1 rows (= fc2 columns), fc1 width, fc2 rows, classes
  int C4;                 // C rounded up to 4
  int M, S, G;            // rows per step (<= 16), steps, workgroups
  int NC, HW;             // fc2 column blocks (G = 8 NC), head workgroups (N2 / 4)
  int nrb, ncb, ntile;    // fc1 row blocks (16 rows), column blocks (256), tiles nrb * ncb
  // device table (int): tile0[G + 1] (workgroup w streams fc1 tiles [tile0[w], tile0[w + 1])
  // in row-major order), then rbw0[nrb] (first workgroup whose run touches each row block),
  // rbn[nrb] (workgroups touching it), hn[NC] (row blocks overlapping each fc2 column block)
  const int* tab;
  const float* X;         // [S * M, K1] inputs (cut activations)
  const int64_t* Y;       // [S * M] labels
  float* loss;            // [S * M] per-row losses
  int64_t ignore;
  float ce_scale;
  SlOpt o;
  const float* adam;      // [S][4] {step_size, inv_bc2_sqrt, CE scale (1 / the step's rows), -}
  const uint32_t* seeds;  // [S][4] {fc1 lo, hi, fc2 lo, hi}
  uint32_t thr1, thr2;
  float dsc1, dsc2;
  int col_off1;           // global index of this shard's fc1 row 0 (dropout hash column)
  // hand-off buffers, double-buffered by step parity, in ONE allocation HB (one buffer
  // resource for all of them); offsets in floats:
  // (the MFMA-produced ones batch-row fastest, [..][n][16 m]: a lane's accumulator is four
  // consecutive rows of one column, so every hand-off store and load is 16 B)
  //   LA [2][nrb][kHySlots][16 n][16 m] look-ahead partials (slot = w - rbw0)
  //   H1 [2][N1][16 m] h1 (rows m >= M zero), written by the F phase's ta == 0 workgroups
  //   FP [2][NC][N2][16 m] fc2 product partials per column block
  //   LP [2][HW][16][C4] logit partials
  //   DL [2][16][C4] dlogits
  //   DZ [2][16][N2] dz2
  //   DP [2][8][N1][16 m] dz1 partials per fc2 row block
  //   ZP [G][kHyRuns][8 waves][64] f32x4 per-wave look-ahead accumulators
  float* HB;
  int oLA, oH1, oFP, oLP, oDL, oDZ, oDP, oZP;
  unsigned* cnt;          // [kHyCounters][kHyStride] (zeroed per launch)
  const int* shard_n;     // [kHySeams][8] arrivals per seam shard and step
  int* err;               // nonzero after a wait gave up (2 timeout, 4 peer exchange)
  int64_t timeout;        // wall-clock ticks per wait
  IpcStep ipc;            // tensor-parallel fc2 exchange (ipc.T == 0: single shard)
  int64_t* trace;         // optional [2][trace_steps][16] phase stamps of workgroups 0 and G - 1
  int trace_steps;
  int64_t* tall;          // optional [tall_n][G][16] phase stamps (as trace) of every workgroup at
  int tall_step, tall_n;  // steps tall_step .. tall_step + tall_n - 1
  int coop;               // cooperative launch (see resident.h)
  int ntst;               // fc1 state policy: over-cache form (1: W plain, m / v non-temporal) or write-through (0)
  int fault_step;         // fault injection (tests): this step's first wait is never met (times out, err 2); -1: off
};

hipError_t hybrid_epoch_launch(const HyArgs& a, hipStream_t st);
int hybrid_lds_bytes();
// shape limits and co-residency of the instantiation the launch would use; why: the reason
std::string hybrid_check(const HyArgs& a);
bool hybrid_fits(const HyArgs& a, int device, std::string* why);

}  // namespace sl
