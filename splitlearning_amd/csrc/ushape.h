// U-shape persistent split epoch (csrc/ushape.hip): every batch of one co-located Alice's
// U-shape epoch -- her conv front (model1) and head (model3), Bob's model2 (fc1 5408 -> N1 ReLU,
// fc2 N1 -> N2 ReLU), the CE on Alice, both backwards and all Adam steps -- in ONE launch, with
// every weight and Adam moment on-chip for the whole epoch (register-resident: fc1's W / m / v
// in VGPRs, fc2 / head / conv in LDS).
#pragma once
#include <string>

#include "common.h"

namespace sl {

constexpr int kUsThreads = 512;   // 8 waves: wave r owns fc1 rows 16 r .. 16 r + 15 of its row group
constexpr int kUsG = 256;         // workgroup w = (row group w >> 5, conv channel w & 31)
constexpr int kUsRG = 8;          // fc1 row groups of 128 rows (= the conv jobs' image pairs)
constexpr int kUsCh = 32;         // conv channels = fc1 column groups (169 columns each)
constexpr int kUsP = 169;         // pooled positions per channel (13 x 13)
constexpr int kUsKB = 11;         // 16-column blocks per channel (169 -> 176, zero padded)
constexpr int kUsKP = 176;
constexpr int kUsN2P = 128;       // fc2 width bound (N2 <= 128)
constexpr int kUsCP = 16;         // head classes bound (C <= 16)
constexpr int kUsW3 = 1024;       // head weights bound (C * N2 <= 1024)
constexpr int kUsStride = 32;     // counter words 128 B apart
// counter words: XC[32] (x slices per channel), PC[8] (fc1 forward partials per row group),
// F2[8] / L[8] / D[8] (fc2 partials / h2 / dlogits, per-XCD shards), DZ[8] (dz1 slices per row
// group), DX[32] (cut-gradient partials per channel), CW[32] (conv gradient partials per channel)
constexpr int kUsXC = 0, kUsPC = 32, kUsF2 = 40, kUsL = 48, kUsD = 56, kUsDZ = 64, kUsDX = 72, kUsCW = 104;
constexpr int kUsFin = 136;       // remote Alice: the launch's closing arrivals (the last dz2's ack)
constexpr int kUsCounters = 137;

// A REMOTE Alice (UsArgs::rem): her conv front and head run in her process (csrc/split.cpp
// run_alice, unchanged) and the launch speaks the peer-mapped channel (csrc/ipc_p2p.h) itself,
// in run_bob's order: per step i it receives her activation (generation rgen0 + 1 + 2 i), sends
// h2 (sgen0 + 1 + 2 i), receives her premasked dz2 (rgen0 + 2 + 2 i) and sends the cut gradient
// (sgen0 + 2 + 2 i), each on the parity slot of its generation.
struct UsLink {
  float* sdata[2];          // her slot data[bob][par]
  uint32_t* sflag[2];       // her flag words [bob][par][chunk]
  const uint32_t* sack[2];  // own ack words [alice][par][chunk]
  const float* rdata[2];    // own slot data[alice][par]
  const uint32_t* rflag[2]; // own flag words [alice][par][chunk]
  uint32_t* rack[2];        // her ack words [bob][par][chunk]
  uint32_t sgen0, rgen0;
  int sprev[2];             // chunk counts of the messages two generations before sends 0 (h2_0), 1 (dx_0)
  int* err;
  int* herr;
};

struct UsArgs {
  // Bob: fc1 [N1][5408], fc2 [N2][N1], Adam moments of each
  float *W1, *m1, *v1, *b1, *mb1, *vb1;
  float *W2, *m2, *v2, *b2, *mb2, *vb2;
  // Alice: conv [32][9] + [32] and head [C][N2] + [C], Adam moments of each
  float *cw, *cb, *cmw, *cmb, *cvw, *cvb;
  float *W3, *m3, *v3, *b3, *mb3, *vb3;
  int N1, N2, C, M, S;
  SlOpt ob, oa;                // Bob's / Alice's Adam (lr, betas, eps, wd; step scalars per step in tabf)
  const float* tabf;           // [S][8] {ss_b, ib_b, ss_a, ib_a, CE scale (1 / the step's rows), rows, -, -}
  const uint8_t* img;          // Alice's shard pixels [N][784]
  const int64_t* rows;         // [S * M] shard row of every batch row (-1: padding)
  const int64_t* Y;            // [S * M] labels (ignore for padding)
  int64_t ignore;
  float* loss;                 // [S * M] per-row losses
  // hand-off buffers in ONE allocation (float offsets), double-buffered by step parity:
  //   XS [2][32 c][16 m][176]          x slices (conv output), columns >= 169 stay zero
  //   PP [2][8 rg][32 c][128 n][16 m]   fc1 forward partials per channel
  //   P2 [2][128 j][256 w][16 m]        fc2 partials per workgroup (its 4 fc1 rows)
  //   H2 [2][128 j][16 m]               h2 (fc2 ReLU output)
  //   DL [2][16 m][16 cls]              dlogits
  //   DZ [2][8 rg][128 n][16 m]         dz1 of each row group
  //   DX [2][32 c][8 rg][176 k][16 m]   cut-gradient partials per row group
  //   CW [2][32 c][8 g][16]             conv gradient partials per image pair
  float* HB;
  int oXS, oPP, oP2, oH2, oDL, oDZ, oDX, oCW;
  unsigned* cnt;               // [kUsCounters][kUsStride] (zeroed per launch)
  int* err;                    // nonzero after a wait gave up (2: timeout)
  int64_t timeout;             // wall-clock ticks per wait
  int coop;
  int bf16;                    // products on bf16 operands (fc1's on bf16 MFMA), fp32 accumulation and state
  int fault_step;              // tests: this step's first wait is never met; -1 off
  // remote Alice: the <.., true> instantiation; RG row groups of 128 fc1 rows, G = 32 RG
  // workgroups (so a one-GPU test can leave CUs to her kernels); tabf [5] = the step's rows
  int rem, RG, G;
  UsLink lk;
};

std::string ushape_check(const UsArgs& a);
bool ushape_fits(const UsArgs& a, int device, std::string* why);
hipError_t ushape_epoch_launch(const UsArgs& a, hipStream_t st);

}  // namespace sl
