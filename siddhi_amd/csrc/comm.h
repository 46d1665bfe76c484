// comm.h -- the multi-GPU exchange of libsiddhi_hip.so (internal interface; the ABI is
// include/siddhi_hip.h sdh_comm_*, sdh_engine_push_bcast, sdh_engine_gather).
//
// One engine per GPU, state private per (pattern, partition key): the path shards with two exchange
// steps and no other collective. Every rank sees the whole event stream (a broadcast of each batch
// from the ingest rank: StreamJunction.sendEvent reaches every subscriber, StreamJunction.java:
// 179-181), and the matches of every rank go to rank 0, where the per-rank runs -- each already in
// the reference's delivery order (R18) -- are merged into the single-engine order on the device.
//
// Two transports behind one protocol:
// * RCCL (ncclCommInitRank from an ncclUniqueId the host distributes): one process per GPU, the
//   deployment; broadcasts, sends and receives run on the engine's stream over xGMI.
// * local: `world` ranks in one process (engines on one or several devices of this process), with
//   the buffers copied device-to-device. The same protocol, so it exercises the gather and merge on
//   one GPU; collectives are one-sided in call order: a broadcast's root pushes first, the other
//   ranks after it (before the root's next push); a gather's non-root ranks call first, rank 0 last.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

struct sdh_comm;

namespace sdh {
namespace xch {

constexpr int HDR = 8;  // int64 words of a protocol header

struct Buf {
  const void* src;  // the sender's device buffer (broadcast root, gather non-root)
  void* dst;        // the receiver's device buffer
  size_t bytes;
};

int rank(const sdh_comm* c);
bool is_local(const sdh_comm* c);
int world(const sdh_comm* c);
int device(const sdh_comm* c);

// Broadcast from `root`: the header (host words, in on the root, out elsewhere), then device
// buffers whose sizes the receivers derive from the header (root: src, dst unused; others: dst).
// Throw std::runtime_error on a transport error, std::invalid_argument on a local-transport call out
// of order.
void bcast_hdr(sdh_comm* c, int64_t hdr[HDR], int root, hipStream_t s);
void bcast_bufs(sdh_comm* c, const std::vector<Buf>& bufs, int root, hipStream_t s);

// Gather to rank 0: every rank's header -- RCCL: an all-gather, every rank receives world x HDR words
// into `all`; local: rank 0 only --, then the buffers (`mine`: src) into rank 0's destinations
// (`recv[r]`: dst). RCCL: every rank passes `mine`, rank 0 its own run too (a self send / receive) and
// recv[0 .. world-1]; local: the non-root ranks pass `mine`, rank 0 recv[1 .. world-1] (its own run
// it copies itself).
void gather_hdr(sdh_comm* c, const int64_t hdr[HDR], int64_t* all, hipStream_t s);
void gather_bufs(sdh_comm* c, const std::vector<Buf>& mine, const std::vector<std::vector<Buf>>& recv, hipStream_t s);

}  // namespace xch
}  // namespace sdh

// k-way merge of k sorted runs on the device (comm.hip). The runs are concatenated: run r is rows
// [run_off[r], run_off[r+1]) of every column; keys hold kw uint64 words per row (most significant
// first), each run sorted by them, ties within a run in run order. off_cat holds each run's ABI
// word offsets (n_r + 1 entries, run-relative) at [run_off[r] + r ...); word_base[r] is where run r's
// words start in `words`. Outputs (N rows, olen / ooff N + 1 entries, osrc / pos N scratch) follow
// include/siddhi_hip.h sdh_matches; *total_words receives ooff[N] once the stream has run.
extern "C" size_t sdh_merge_temp_bytes(int64_t n);
extern "C" hipError_t sdh_merge_runs(const uint64_t* keys, int kw, const int64_t* run_off, int k, int64_t N,
                                     const int64_t* q, const int64_t* key, const int64_t* ts, const int64_t* seq,
                                     const int64_t* tb, const int64_t* off_cat, const int64_t* word_base,
                                     int64_t* pos, int64_t* oq, int64_t* okey, int64_t* ots, int64_t* oseq,
                                     int64_t* otb, int64_t* olen, int64_t* ooff, int64_t* osrc, void* temp,
                                     size_t temp_bytes, int64_t* total_words, hipStream_t s);
extern "C" hipError_t sdh_merge_words(const int64_t* osrc, const int64_t* ooff, int64_t N, const int64_t* words,
                                      int64_t* owords, hipStream_t s);
