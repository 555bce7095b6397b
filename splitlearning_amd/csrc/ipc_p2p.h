// Point-to-point messages over peer-mapped HBM (`_C.IpcChannel`): the split-mode data plane
// (activation + labels to Bob, cut gradient back; U-shape also the middle output and its
// gradient) between two processes, issued from C++ on the compute stream.
//
// Why: the split modes move 2 - 4 latency-bound messages per batch.  RCCL cannot pair two
// ranks on one GPU at all (the --ranks_share_gpu rehearsal), and across GPUs an ncclSend /
// ncclRecv pair is a proxy-driven protocol with its own launch per call.  Here every rank
// exports one receive region (uncached device memory) and maps every peer's once; a send is
// ONE kernel on the sender that writes the message straight into the receiver's region over
// the xGMI link (one hop) and raises a per-chunk flag, a receive is ONE kernel that waits on
// its own flags and copies the message out.
//
// Protocol (per ordered pair s -> d, generation g = the pair's message count, kept by both
// sides in program order):
//   sender s, workgroup c (chunk c of kIpcChunk floats):
//     wait ack[d][par][c] >= g - 2 in ITS OWN region (d has read what the slot held two
//     messages ago; parity par = g & 1 double-buffers the slot) ->
//     16-B write-through stores of the chunk into d's data[s][par] -> drain -> release ->
//     flag[s][par][c] = g in d's region;
//   receiver d, workgroup c:
//     wait flag[s][par][c] >= g in its own region -> acquire -> copy the chunk out -> drain ->
//     ack[d][par][c] = g in s's region.
// Memory ordering as ipc_ar.h (system scope, release before the flag, acquire after it).
// Every wait is bounded by wall clock; a timeout raises the error word (and its host-pinned
// mirror) and every later wait on this rank gives up at once, so a dead peer costs one
// timeout and the job reads the word at the end of the epoch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "ipc_ar.h"

namespace sl {

// One message's view of the regions, handed to the send / receive kernel
struct P2PMsg {
  float* data;          // send: the receiver's slot data[me][par]; recv: own slot data[src][par]
  uint32_t* flag;       // send: the receiver's flag[me][par][0..]; recv: own flag[src][par][0..]
  uint32_t* ack;        // send: own ack[dst][par][0..];           recv: the sender's ack[me][par][0..]
  uint32_t gen;
  int* err;
  int* herr;
  int64_t timeout;      // wall-clock ticks
};

// The pair's regions and generations handed to a persistent kernel that sends and receives a
// run of messages itself (csrc/vanilla.hip's remote-Alice epoch): send j of the run carries
// generation sgen0 + 1 + j, receive j rgen0 + 1 + j, each on the slot of its generation's parity
struct P2PRun {
  float* sdata[2];
  uint32_t* sflag[2];
  uint32_t* sack[2];
  float* rdata[2];
  uint32_t* rflag[2];
  uint32_t* rack[2];
  uint32_t sgen0, rgen0;
  int sprev[2];        // chunk counts of the messages two generations before sends 0 and 1
  int* err;
  int* herr;
  int64_t timeout;
};

class IpcChannel {
 public:
  // cap: the largest message (floats) this channel carries
  IpcChannel(int nranks, int rank, int64_t cap);
  ~IpcChannel();
  IpcChannel(const IpcChannel&) = delete;
  IpcChannel& operator=(const IpcChannel&) = delete;
  std::string handle() const;
  void open(const std::vector<std::string>& handles);
  // n floats from x (16-B aligned, n % 4 == 0, n <= cap) to / from rank `peer`, on stream st.
  // Stream-ordered; every call of a pair advances that pair's generation on both sides.  All
  // sends to one peer must be issued on ONE stream, and all receives from one peer on one
  // stream: a chunk beyond the previous message's chunk count waits on chunk 0's ack, which
  // is only ordered after that message's receive if the receives are stream-ordered.  The
  // first call binds the stream; a call on another stream throws.
  void send(const float* x, int64_t n, int peer, hipStream_t st);
  void recv(float* x, int64_t n, int peer, hipStream_t st);
  // A run of messages with `peer` that ONE kernel on stream st sends / receives itself: the
  // floats of each send and receive, in issue order.  Checks them as send / recv would, binds
  // the streams, and advances the pair's generations and slot history exactly as that many
  // send / recv calls, so the channel's later messages continue the sequence.
  P2PRun run(int peer, hipStream_t st, const std::vector<int64_t>& sends, const std::vector<int64_t>& recvs);
  bool serves(const void* p, int64_t n) const {
    return n <= cap_ && n % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  }
  int error() const;
  int host_error() const { return __atomic_load_n(herr_, __ATOMIC_ACQUIRE); }
  void set_timeout_s(double s) { timeout_ = (int64_t)(s * 1000.0 * clock_khz_); }
  double timeout_s() const { return (double)timeout_ / (1000.0 * clock_khz_); }
  int64_t cap() const { return cap_; }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool opened() const { return opened_; }
  uint32_t sent(int peer) const { return send_gen_.at(peer); }
  uint32_t received(int peer) const { return recv_gen_.at(peer); }

 private:
  // region layout (floats / words): data [T src][2][cap]; sync words [2 kinds][T][2][nch]
  // (kind 0 flags indexed by the source, kind 1 acks indexed by the destination)
  void check(const void* x, int64_t n, int peer) const;
  int64_t flag_off(int src, int par) const { return ((int64_t)src * 2 + par) * nch_; }
  int64_t ack_off(int dst, int par) const { return ((int64_t)(nranks_ + dst) * 2 + par) * nch_; }
  int nranks_, rank_;
  int64_t cap_;
  int nch_;
  float* data_ = nullptr;
  uint32_t* syncw_ = nullptr;
  int* err_ = nullptr;
  int* herr_ = nullptr;
  int* herr_dev_ = nullptr;
  float* peer_data_[kIpcMaxRanks] = {};
  uint32_t* sync_[kIpcMaxRanks] = {};
  std::vector<void*> mapped_;
  std::vector<uint32_t> send_gen_, recv_gen_;
  std::vector<int> hist_;      // [peer][parity]: chunk count of the last message sent on it
  std::vector<hipStream_t> send_st_, recv_st_;   // the stream bound per peer (first call)
  std::vector<char> send_bound_, recv_bound_;
  void bind_stream(std::vector<hipStream_t>& sts, std::vector<char>& bound, int peer, hipStream_t st,
                   const char* what);
  bool opened_ = false;
  int64_t timeout_ = 0;
  int clock_khz_ = 100000;
};

}  // namespace sl
