// Vanilla persistent split epoch (csrc/vanilla.hip): every batch of one co-located Alice's
// vanilla epoch -- her conv front (forward, backward, SGD-momentum) AND Bob's whole 3-layer
// tail (forward, CE, backward, SGD-momentum, the cut gradient) -- in ONE cooperative launch.
// Bob's fc2 / fc3 and the biases stay on-chip (as csrc/hybrid.hip); fc1's W / momentum
// stream twice per step: an update pass that also forms the cut gradient from the old
// weights, and a forward pass of the next batch over the updated ones.
#pragma once
#include "common.h"
#include "resident.h"

namespace sl {

constexpr int kVaThreads = 512;     // one 8-wave workgroup per CU
constexpr int kVaG = 256;           // workgroups (one per CU): 32 conv channels x 8 image pairs
constexpr int kVaNR = 8;            // fc2 row blocks
constexpr int kVaMaxNC = 32;        // fc2 column blocks (G = 8 NC)
constexpr int kVaMaxWR = 128;       // fc2 tile rows
constexpr int kVaMaxWC4 = 40;       // fc2 tile columns / 4
constexpr int kVaMaxC = 128;        // classes
constexpr int kVaRuns = 3;          // fc1 row blocks one forward-pass run may touch
constexpr int kVaSlots = 8;         // workgroups whose forward runs may touch one fc1 row block
constexpr int kVaMaxRB = 320;       // fc1 row blocks of 16 rows (N1 <= 5120)
constexpr int kVaMaxCB = 24;        // fc1 column blocks of 256 (K1 <= 6144)
constexpr int kVaMaxRun = 28;       // update-pass run length (tiles)
constexpr int kVaDxSlots = 16;      // workgroups whose update runs may touch one column block
constexpr int kVaStride = 32;       // counter words 128 B apart
constexpr int kVaSeams = 5;         // F: fc2 partials, L: logit partials, D: dlogits, Z: dz2, X: next batch
// counter words: the seams' 8 shards each, then P[NC] (dz1 partials per fc2 column block),
// R[nrb] (forward partials per fc1 row block), XD[ncb] (cut-gradient partials per fc1 column
// block), CW[32] (conv gradient partials per channel), CX[32] (next-batch activations per channel)
constexpr int kVaMaxS = 6000;      // steps per launch (the activation slots' 32-bit offsets)
constexpr int kVaCounters = kVaSeams * 8 + kVaMaxNC + kVaMaxRB + kVaMaxCB + 32 + 32;

// A REMOTE Alice (VaArgs::rem): her conv front runs in her own process (csrc/split.cpp
// run_alice, unchanged) and the launch speaks the peer-mapped channel's protocol
// (csrc/ipc_p2p.h) itself: per step i it receives her activation message of step i (generation
// rgen0 + 1 + i) and sends her the cut gradient of step i (generation sgen0 + 1 + i), each on
// the parity slot of its generation -- the same messages, sizes and order as run_bob.
struct VaLink {
  float* sdata[2];          // her slot data[bob][par]: the cut gradients land there
  uint32_t* sflag[2];       // her flag words [bob][par][chunk]
  const uint32_t* sack[2];  // own ack words [alice][par][chunk] (she acks a cut gradient read)
  const float* rdata[2];    // own slot data[alice][par]: her activation messages
  const uint32_t* rflag[2]; // own flag words [alice][par][chunk]
  uint32_t* rack[2];        // her ack words [bob][par][chunk] (acks of her activations)
  uint32_t sgen0, rgen0;    // the pair's generations before the launch's first message
  int sprev[2];             // chunk counts of the messages sent two generations before sends 0, 1
  int* err;                 // the channel's error word (uncached) and its host-pinned mirror
  int* herr;
};

struct VaArgs {
  ResLayer L1, L2, L3;    // Bob's tail (v unused: SGD-momentum)
  int N1, K1, N2, C, C4;  // fc1 rows, fc1 width (5408), fc2 rows, classes, C rounded up to 4
  int M, S, G;            // rows per step (<= 16), steps, workgroups
  int NC, HW;             // fc2 column blocks (G = 8 NC), head workgroups (N2 / 4)
  int nrb, ncb, ntile;    // fc1 row blocks, column blocks, tiles
  // device table (int): the forward pass's row-major runs as hybrid.h (tile0[G + 1], rbw0[nrb],
  // rbn[nrb], hn[NC]), then the update pass's runs: cbn[ncb] (workgroups touching the column
  // block) at oU; per workgroup {v0, v1, rb0, nb} at oUW: its run [v0, v1) of the row band
  // [rb0, rb0 + nb) walked column-major (tile v: column block v / nb, row block rb0 + v % nb);
  // per workgroup and column block its dx slot (-1: untouched) at oUS ([G][ncb])
  const int* tab;
  int oU, oUW, oUS;
  // Alice: uint8 shard pixels [N, 784], the batch rows of every step ([S * M] shard row
  // indices, -1 = padding), her conv weights / bias and their momentum buffers
  const uint8_t* img;
  const int64_t* rows;
  float *cw, *cb, *cmw, *cmb;
  SlOpt oa;               // Alice's optimizer (SGD-momentum)
  const int64_t* Y;       // [S * M] labels (ignore for padding rows)
  float* loss;            // [S * M] per-row losses
  int64_t ignore;
  SlOpt o;                // Bob's optimizer (SGD-momentum)
  const float* adam;      // [S][4] {the step's rows, -, CE scale (1 / the step's rows), -}
  const uint32_t* seeds;  // [S][4] {fc1 lo, hi, fc2 lo, hi}
  uint32_t thr1, thr2;
  float dsc1, dsc2;
  // hand-off buffers in ONE allocation HB (offsets in floats), MFMA-produced ones batch-row
  // fastest as hybrid.h:
  //   LA [2][nrb][kVaSlots][16 n][16 m] forward partials    H1 [2][N1][16 m] h1
  //   FP [2][NC][N2][16 m] fc2 partials                      LP [2][HW][16][C4] logit partials
  //   DL [2][16][C4] dlogits                                 DZ [2][16][N2] dz2
  //   DP [2][8][N1][16 m] dz1 partials
  //   DX [ncb][kVaDxSlots][16 m][256] cut-gradient partials
  //   CWP [2][32][8][16] conv gradient partials per (channel, image pair)
  // the batches' activations, one [16][K1] slot per step of the launch (each written once,
  // before any read; read with sc1 loads like every handed-off byte)
  float* Xr;
  float* HB;
  int oLA, oH1, oFP, oLP, oDL, oDZ, oDP, oDX, oCWP;
  unsigned* cnt;          // [kVaCounters][kVaStride] (zeroed per launch)
  const int* shard_n;     // [kVaSeams][8] arrivals per seam shard and step
  int* err;               // nonzero after a wait gave up (2 timeout)
  int64_t timeout;        // wall-clock ticks per wait
  int coop;               // cooperative launch
  int fault_step;         // tests: this step's first wait is never met; -1 off
  int64_t* tall;          // optional [tall_n][G][16] phase stamps (wall clock) of every workgroup
  int tall_step, tall_n;  // for steps tall_step .. tall_step + tall_n - 1
  // remote Alice: the kernel's <true> instantiation; no conv jobs, so G may be any multiple of
  // 8 up to 256 that the fc2 tiling allows (a one-GPU test leaves CUs to the Alice's kernels).
  // Yrem: the launch-local [S * M] labels the kernel fills from the messages (Y unused).
  int rem;
  int64_t* Yrem;
  VaLink lk;
};

hipError_t vanilla_epoch_launch(const VaArgs& a, hipStream_t st);
int vanilla_lds_bytes();
std::string vanilla_check(const VaArgs& a);
bool vanilla_fits(const VaArgs& a, int device, std::string* why);

}  // namespace sl
