// matches.hip -- the device match table and the R18-ordered poll.
//
// The reference delivers every completed StateEvent to QuerySelector.process one at a time, in the
// order R18 fixes: per input event (StreamJunction.java:179-181), per receiver / query, per state
// processor in reverse registration order, per pending partial in insertion order
// (StateMultiProcessStreamReceiver.java:53-74, SingleProcessStreamReceiver.java:57-80). The kernels
// emit out of that order (lanes, chunks and keys run in parallel), so each push appends its matches
// to a device table together with their R18 sort keys (nfa_types.h MatchTable), and a poll sorts the
// table on the device -- stable LSD radix passes over the tiebreak keys, then the (trigger seq,
// out_rank) key -- and gathers the ABI tuples of include/siddhi_hip.h (query, key, ts, off, words)
// in HBM. sdh_engine_poll copies them to the host; sdh_engine_poll_device hands them out in place.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "nfa_types.h"

namespace sdh {

namespace {

__device__ __forceinline__ uint64_t hi_key(int64_t seq, int64_t seq_ref, int rank) {
  return ((uint64_t)(seq - seq_ref) << RANK_BITS) | (uint64_t)rank;
}

// K_ratchet blocks (nfa_ratchet.hip record format) -> table rows; one workgroup per block
__global__ __launch_bounds__(256) void append_ratchet_kernel(
    const int64_t* __restrict__ match, int blk_recs, int wide, const int32_t* __restrict__ blk_count,
    const int32_t* __restrict__ blk_group, const int64_t* __restrict__ dst_off, const RatchetGroup* __restrict__ groups,
    const int64_t* __restrict__ ts, int64_t seq_base, int64_t seq_ref, const int32_t* __restrict__ out_rank,
    int n_streams, MatchTable T, int64_t row0, int64_t word0) {
  const int b = blockIdx.x;
  const int n = blk_count[b];
  const RatchetGroup* G = groups + blk_group[b];
  const uint2* R = reinterpret_cast<const uint2*>(match) + ((size_t)b * blk_recs << (wide ? 1 : 0));
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t off, ln, q1;
    if (!wide) {
      const uint2 r = R[i];
      off = r.x & ((1u << 26) - 1);
      ln = r.x >> 26;
      q1 = r.y;
    } else {
      const uint4 r = reinterpret_cast<const uint4*>(R)[i];
      off = r.x;
      ln = r.y & 63;
      q1 = r.z;
    }
    const int64_t s = seq_base + (int64_t)off;
    const int64_t s1 = s - (int64_t)(uint32_t)((uint32_t)s - q1);
    const int q = G->qid[ln];
    const int64_t row = row0 + dst_off[b] + i;
    const int64_t w = word0 + (row - row0) * 4;
    T.hi[row] = hi_key(s, seq_ref, out_rank[(int64_t)q * n_streams + G->stream]);
    T.lo[0][row] = (uint64_t)s1;
#pragma unroll
    for (int k = 1; k < MAXLO; ++k) T.lo[k][row] = 0ull;
    T.seq[row] = s;
    T.q[row] = q;
    T.key[row] = -1;
    T.ts[row] = ts[off];
    T.woff[row] = w;
    T.wlen[row] = 4;
    reinterpret_cast<longlong2*>(T.words + w)[0] = make_longlong2(1, s1);
    reinterpret_cast<longlong2*>(T.words + w)[1] = make_longlong2(1, s);
  }
}

// One K_ratchet record of block b (nfa_types.h RatchetLaunch; include/siddhi_hip.h sdh_records):
// its e2 batch offset, lane and the low 32 bits of e1's seq. ns >= 0: a rec4 block of ns side entries
// (entry i's event is the last side entry whose first index is <= i; side entry j sits at byte
// blk_recs * 8 - 8 * (j + 1)).
__device__ __forceinline__ void ratchet_record(const int64_t* match, int blk_recs, int wide, int b, int ns, int i,
                                               uint32_t sb32, uint32_t& off, uint32_t& ln, uint32_t& q1) {
  const char* B = reinterpret_cast<const char*>(match) + ((size_t)b * blk_recs * 8 << (wide ? 1 : 0));
  if (ns >= 0) {
    const uint32_t* E = reinterpret_cast<const uint32_t*>(B);
    const uint2* S = reinterpret_cast<const uint2*>(B + (size_t)blk_recs * 8);  // S[-1 - j] = side entry j
    int lo = 0, hi = ns - 1;  // side entry 0's first index is 0 <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int)S[-1 - mid].x <= i) lo = mid;
      else hi = mid - 1;
    }
    off = S[-1 - lo].y;
    ln = E[i] >> 26;
    q1 = (sb32 + off) - (E[i] & ((1u << 26) - 1));
  } else if (!wide) {
    const uint2 r = reinterpret_cast<const uint2*>(B)[i];
    off = r.x & ((1u << 26) - 1);
    ln = r.x >> 26;
    q1 = r.y;
  } else {
    const uint4 r = reinterpret_cast<const uint4*>(B)[i];
    off = r.x;
    ln = r.y & 63;
    q1 = r.z;
  }
}

// Order-independent digest of the K_ratchet records of the last launch (both output modes write the
// same per-wave blocks): per record mix64(e2 seq, query, e1 seq) summed mod 2^64, and the record count.
// Test diagnostics (sdh_engine_debug_digest): normal and device-record modes must write the same records.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void digest_ratchet_kernel(const int64_t* __restrict__ match, int blk_recs, int wide,
                                                             const int32_t* __restrict__ blk_count,
                                                             const int32_t* __restrict__ blk_group,
                                                             const int32_t* __restrict__ blk_side,
                                                             const RatchetGroup* __restrict__ groups, int64_t seq_base,
                                                             unsigned long long* acc) {
  const int b = blockIdx.x;
  const int n = blk_count[b];
  const int ns = blk_side[b];  // >= 0: a rec4 block (nfa_types.h RatchetLaunch::rec4)
  const RatchetGroup* G = groups + blk_group[b];
  unsigned long long h = 0, c = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t off, ln, q1;
    ratchet_record(match, blk_recs, wide, b, ns, i, (uint32_t)seq_base, off, ln, q1);
    const int64_t s = seq_base + (int64_t)off;
    const int64_t s1 = s - (int64_t)(uint32_t)((uint32_t)s - q1);
    h += mix64(mix64((uint64_t)s * 0x9E3779B97F4A7C15ull ^ (uint64_t)G->qid[ln]) ^ (uint64_t)s1);
    ++c;
  }
  for (int o = 32; o > 0; o >>= 1) {
    h += __shfl_down(h, o);
    c += __shfl_down(c, o);
  }
  if ((threadIdx.x & 63) == 0 && c) {
    atomicAdd(&acc[0], c);
    atomicAdd(&acc[1], h);
  }
}

// Device records -> compact rows (sdh_engine_records_compact): block b's records at rows
// row_off[b] .. row_off[b] + blk_count[b] (an exclusive scan of blk_count), each
// {query, e2 - seq_base, e2 - e1, 0, INT32_MIN...} of `width` int32 (the sdh_matches_compact form)
__global__ __launch_bounds__(256) void ratchet_compact_kernel(const int64_t* __restrict__ match, int blk_recs, int wide,
                                                              const int32_t* __restrict__ blk_count,
                                                              const int32_t* __restrict__ blk_group,
                                                              const int32_t* __restrict__ blk_side,
                                                              const RatchetGroup* __restrict__ groups,
                                                              const int64_t* __restrict__ row_off, int64_t seq_base,
                                                              int width, int32_t* __restrict__ rows) {
  const int b = blockIdx.x;
  const int n = blk_count[b];
  const int ns = blk_side[b];
  const RatchetGroup* G = groups + blk_group[b];
  const int64_t r0 = row_off[b];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t off, ln, q1;
    ratchet_record(match, blk_recs, wide, b, ns, i, (uint32_t)seq_base, off, ln, q1);
    int32_t* o = rows + (r0 + i) * width;
    const int32_t d = (int32_t)((uint32_t)(seq_base + off) - q1);
    if (width == 4) {
      *reinterpret_cast<int4*>(o) = make_int4(G->qid[ln], (int32_t)off, d, 0);
    } else {
      o[0] = G->qid[ln];
      o[1] = (int32_t)off;
      o[2] = d;
      o[3] = 0;
      for (int j = 4; j < width; ++j) o[j] = INT32_MIN;
    }
  }
}

// ---- K_ratchet direct R18 placement (a push whose matches all come from K_ratchet) ----
// nfa_ratchet.hip's COUNT pass stores each (event, group) match total, an exclusive scan over them
// (sdh_place_scan) gives each cell's first row, and the WRITE pass writes every match as its
// COMPACT row (sdh_matches_compact) at its R18 row: no records, no sort. The ABI columns are built
// from the compact rows only when a poll asks for the full tuples (compact_fill_kernel).

// compact rows of a placed window (K_ratchet: two one-event slots) -> the ABI columns of rows
// [0, rows): words {1, e1, 1, e2} per row, ts from the window's event-time log (ts_log[seq - seq_ref])
__global__ __launch_bounds__(256) void compact_fill_kernel(const int32_t* __restrict__ crow, int width, int64_t rows,
                                                           const int64_t* __restrict__ ts_log, int64_t seq_ref,
                                                           int64_t* __restrict__ oq, int64_t* __restrict__ okey,
                                                           int64_t* __restrict__ ots, int64_t* __restrict__ oseq,
                                                           int64_t* __restrict__ otb, int64_t* __restrict__ ooff,
                                                           int64_t* __restrict__ owords) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > rows) return;
  if (i == rows) {
    ooff[rows] = 4 * rows;
    return;
  }
  const int32_t* r = crow + i * width;
  const int64_t e2 = seq_ref + (int64_t)r[1], e1 = e2 - (int64_t)r[2];
  oq[i] = r[0];
  okey[i] = -1;
  ots[i] = ts_log[r[1]];
  oseq[i] = e2;
  otb[i] = INT64_MIN;
  ooff[i] = 4 * i;
  reinterpret_cast<longlong2*>(owords + 4 * i)[0] = make_longlong2(1, e1);
  reinterpret_cast<longlong2*>(owords + 4 * i)[1] = make_longlong2(1, e2);
}

// placed compact rows [0, n) -> general table rows (a later push in the same poll window has other
// producers)
__global__ __launch_bounds__(256) void placed_to_table_kernel(const int32_t* __restrict__ crow, int width, int64_t n,
                                                              const int64_t* __restrict__ ts_log, int64_t seq_ref,
                                                              const int32_t* __restrict__ out_rank,
                                                              const int32_t* __restrict__ qinfo, int n_streams,
                                                              MatchTable T) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t* r = crow + i * width;
  const int qq = r[0];
  const int64_t e2 = seq_ref + (int64_t)r[1], e1 = e2 - (int64_t)r[2];
  T.hi[i] = hi_key(e2, seq_ref, out_rank[(int64_t)qq * n_streams + qinfo[2 * qq + 1]]);
  T.lo[0][i] = (uint64_t)e1;
#pragma unroll
  for (int k = 1; k < MAXLO; ++k) T.lo[k][i] = 0ull;
  T.seq[i] = e2;
  T.q[i] = qq;
  T.key[i] = -1;
  T.ts[i] = ts_log[r[1]];
  T.woff[i] = 4 * i;
  T.wlen[i] = 4;
  reinterpret_cast<longlong2*>(T.words + 4 * i)[0] = make_longlong2(1, e1);
  reinterpret_cast<longlong2*>(T.words + 4 * i)[1] = make_longlong2(1, e2);
}

// R18-sorted table rows -> compact rows (sdh_engine_poll_compact on a window with other producers):
// [query, trigger seq - seq_ref, per slot trigger seq - its event's seq (INT32_MIN: empty)].
// err[0] = 1 when a row does not fit the form: a slot with a chain of several events (count
// states), a partition key, a timer match, or a seq distance past int32.
__global__ __launch_bounds__(256) void table_compact_kernel(MatchTable T, const int32_t* __restrict__ perm, int64_t n,
                                                            int width, int64_t seq_ref, int32_t* __restrict__ crow,
                                                            int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t p = perm[i];
  int32_t* o = crow + i * width;
  const int64_t sq = T.seq[p];
  bool bad = T.key[p] != -1 || (T.hi[p] & ((1ull << RANK_BITS) - 1)) == 0 || sq - seq_ref > INT32_MAX;
  o[0] = (int32_t)T.q[p];
  o[1] = (int32_t)(sq - seq_ref);
  const int64_t* w = T.words + T.woff[p];
  const int64_t len = T.wlen[p];
  int slot = 0;
  for (int64_t j = 0; j < len && !bad; ++slot) {
    const int64_t c = w[j];
    if (c > 1 || 2 + slot >= width) {
      bad = true;
      break;
    }
    const int64_t d = c == 1 ? sq - w[j + 1] : 0;
    if (d < 0 || d > INT32_MAX) bad = true;
    o[2 + slot] = c == 1 ? (int32_t)d : INT32_MIN;
    j += 1 + c;
  }
  for (int k = 2 + slot; k < width; ++k) o[k] = INT32_MIN;
  if (bad) atomicOr(err, 1);
}

// K_chain segments (records {qid, ts, seq_0 .. seq_{S-1}} of rec_words) -> table rows
__global__ __launch_bounds__(256) void append_chain_kernel(
    const int64_t* __restrict__ src, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_count,
    const int64_t* __restrict__ dst_off, int rec_words, const int32_t* __restrict__ qinfo, int64_t seq_ref,
    const int32_t* __restrict__ out_rank, int n_streams, MatchTable T, int64_t row0, int64_t word0) {
  const int item = blockIdx.x;
  const int64_t n = seg_count[item];
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t* v = src + (seg_off[item] + i) * rec_words;
    const int q = (int)v[0];
    const int S = qinfo[2 * q], last_stream = qinfo[2 * q + 1];
    const int64_t row = row0 + dst_off[item] + i;
    const int64_t w = word0 + (row - row0) * 2 * MAXS;
    T.hi[row] = hi_key(v[2 + S - 1], seq_ref, out_rank[(int64_t)q * n_streams + last_stream]);
    T.seq[row] = v[2 + S - 1];
#pragma unroll
    for (int k = 0; k < MAXLO; ++k) T.lo[k][row] = k < S - 1 ? (uint64_t)v[2 + k] : 0ull;
    T.q[row] = q;
    T.key[row] = -1;
    T.ts[row] = v[1];
    T.woff[row] = w;
    T.wlen[row] = 2 * S;
    for (int k = 0; k < S; ++k) {
      T.words[w + 2 * k] = 1;
      T.words[w + 2 * k + 1] = v[2 + k];
    }
  }
}

// The table words each record of a push takes (tw[n_rec] = 0, for the exclusive scan): a K_gen / K_seq
// record [len, qid, key, ts, seq, idx, S | stream << 16, (count, seqs...) x S] its slot words, a
// narrow K_part or K_seq record (nfa_types.h) its slots expanded to that form
__device__ __forceinline__ int32_t lo32(int64_t w) { return (int32_t)(uint32_t)(uint64_t)w; }
__device__ __forceinline__ int32_t hi32(int64_t w) { return (int32_t)(uint32_t)((uint64_t)w >> 32); }

__global__ __launch_bounds__(256) void gen_rec_words_kernel(const int64_t* __restrict__ out,
                                                            const int64_t* __restrict__ rec_off, int64_t n_rec,
                                                            int64_t* __restrict__ tw, unsigned long long* n_wide) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_rec) return;
  if (i == n_rec) {
    tw[i] = 0;
    return;
  }
  const int64_t* r = out + rec_off[i];
  const int32_t l0 = lo32(r[0]);
  if (l0 >= 0) {
    tw[i] = r[0] - 7;
    atomicAdd(n_wide, 1ull);
  } else if (((-l0) >> 16) == NREC_KIND_COUNT) {  // count: (1, e1), (c, chain), (1, trigger)
    tw[i] = 5 + hi32(r[2]);
  } else if (((-l0) >> 16) == NREC_KIND_SEQ) {    // K_seq window: (1, seq) x S
    tw[i] = 2 * hi32(r[1]);
  } else {  // or / and: (1, e1), then per side (1, seq) or (0)
    tw[i] = 2 + (hi32(r[2]) == INT32_MIN ? 1 : 2) + (lo32(r[3]) == INT32_MIN ? 1 : 2);
  }
}

// the push's records -> table rows, each row's words at word0 + woff[i] (gen_rec_words_kernel, scanned).
// Narrow records take the trigger's ts from the batch (bts[offset]), their key from the partition's key
// table (qkeys[query][key id]) and e1's seq as the emission index.
__global__ __launch_bounds__(256) void append_gen_kernel(const int64_t* __restrict__ out,
                                                         const int64_t* __restrict__ rec_off, int64_t n_rec,
                                                         int64_t seq_ref, const int32_t* __restrict__ out_rank,
                                                         const int32_t* __restrict__ fan_rank, int n_streams,
                                                         MatchTable T, int64_t row0, int64_t word0,
                                                         const int64_t* __restrict__ woff,
                                                         const int64_t* __restrict__ bts, int64_t seq_base,
                                                         int bstream, const int64_t* const* __restrict__ qkeys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rec) return;
  const int64_t* r = out + rec_off[i];
  const int64_t row = row0 + i;
  const int64_t wo = word0 + woff[i];
  int64_t* w = T.words + wo;
  T.woff[row] = wo;
  static_assert(MAXLO >= 3, "timer tiebreaks");
  const int32_t l0 = lo32(r[0]);
  if (l0 < 0 && ((-l0) >> 16) == NREC_KIND_SEQ) {  // narrow K_seq record
    const int q = hi32(r[0]), S = hi32(r[1]);
    const int64_t off = (int64_t)(uint32_t)lo32(r[1]);
    const int64_t sq = seq_base + off;
    T.seq[row] = sq;
    T.hi[row] = hi_key(sq, seq_ref, out_rank[(int64_t)q * n_streams + bstream]);
    T.lo[0][row] = 0ull;  // (one match per event and query)
    T.lo[1][row] = 0ull;
    T.lo[2][row] = 0ull;
    T.q[row] = q;
    T.key[row] = -1;
    T.ts[row] = bts[off];
    for (int j = 0; j < S - 1; ++j) {
      w[2 * j] = 1;
      w[2 * j + 1] = sq - (j & 1 ? hi32(r[2 + j / 2]) : lo32(r[2 + j / 2]));
    }
    w[2 * S - 2] = 1;
    w[2 * S - 1] = sq;
    T.wlen[row] = 2 * S;
    return;
  }
  if (l0 < 0) {  // narrow K_part record
    const bool count = ((-l0) >> 16) == NREC_KIND_COUNT;
    const int q = hi32(r[0]);
    const int64_t off = (int64_t)(uint32_t)lo32(r[1]);
    const uint32_t kid = (uint32_t)hi32(r[1]);
    const int64_t sq = seq_base + off, e1 = sq - lo32(r[2]);
    T.seq[row] = sq;
    T.hi[row] = hi_key(sq, seq_ref, out_rank[(int64_t)q * n_streams + bstream]);
    T.lo[0][row] = (uint64_t)e1;
    T.lo[1][row] = 0ull;
    T.lo[2][row] = 0ull;
    T.q[row] = q;
    T.key[row] = qkeys[q][kid];
    T.ts[row] = bts[off];
    int k = 0;
    w[k++] = 1;
    w[k++] = e1;
    if (count) {
      const int c = hi32(r[2]);
      w[k++] = c;
      for (int j = 0; j < c; ++j) w[k++] = sq - (j & 1 ? hi32(r[3 + j / 2]) : lo32(r[3 + j / 2]));
      w[k++] = 1;
      w[k++] = sq;
    } else {
      for (int s = 0; s < 2; ++s) {
        const int32_t d = s == 0 ? hi32(r[2]) : lo32(r[3]);
        if (d == INT32_MIN) {
          w[k++] = 0;
        } else {
          w[k++] = 1;
          w[k++] = sq - d;
        }
      }
    }
    T.wlen[row] = k;
    return;
  }
  const int q = (int)r[1], stream = (int)((r[6] >> 16) & 0xFFFF);
  T.seq[row] = r[4];
  if (stream == 0xFFFF) {
    // an absent state's timer match (nfa_gen.hip): rank 0, before the trigger event's own matches;
    // then by (timer key, query, partition key) -- later lo passes are more significant -- and one
    // instance's matches keep their emission order (the sort is stable, rows are appended in it)
    T.hi[row] = hi_key(r[4], seq_ref, 0);
    T.lo[2][row] = (uint64_t)r[5] ^ 0x8000000000000000ull;
    T.lo[1][row] = (uint64_t)(uint32_t)q;
    T.lo[0][row] = (uint64_t)r[2] ^ 0x8000000000000000ull;
  } else if (fan_rank && fan_rank[(int64_t)q * n_streams + stream] >= 0) {
    // a fan-out stream's match (PartitionStreamReceiver.send(ComplexEvent)): the partition's
    // rank, then the key's junction-map position, the query's rank in the partition, emission
    T.hi[row] = hi_key(r[4], seq_ref, out_rank[(int64_t)q * n_streams + stream]);
    T.lo[2][row] = (uint64_t)r[5] >> 32;
    T.lo[1][row] = (uint64_t)fan_rank[(int64_t)q * n_streams + stream];
    T.lo[0][row] = (uint64_t)r[5] & 0xFFFFFFFFull;
  } else {
    T.hi[row] = hi_key(r[4], seq_ref, out_rank[(int64_t)q * n_streams + stream]);
    T.lo[0][row] = (uint64_t)r[5];
    T.lo[1][row] = 0ull;
    T.lo[2][row] = 0ull;
  }
  T.q[row] = q;
  T.key[row] = r[2];
  T.ts[row] = r[3];
  const int64_t len = r[0] - 7;
  T.wlen[row] = len;
  for (int64_t k = 0; k < len; ++k) w[k] = r[7 + k];
}

// Chunk delivery keys (nfa_types.h MatchTable chi / clo) of rows [r0, r1).
// chunk == 0: single-event rows -- chi = their hi with the rank cleared, clo = 0, so the final
// (chi, clo) passes keep their (seq, rank, tiebreak) order.
// chunk != 0: rows of a chunk push over stream `stream` whose first event has seq first_seq. The
// reference hands the whole chunk to one junction subscriber after another; a partition splits it
// into same-key runs (each run to every clone of its key, one clone after another) or, for a stream
// it does not key, gives all of it to every key in junction-map order; inside a clone the events
// go in order. So a row sorts by (chunk, subscriber rank major[q], run start runs[slot][event] or
// key position lo[2] (fan-out rows, append_gen_kernel), its query's rank in the partition minor[q],
// then its single-event key). Timer rows (rank 0: fired before the chunk) come first.
__global__ void chunk_keys_kernel(MatchTable T, int64_t r0, int64_t r1, int chunk, int64_t cseq, int64_t first_seq,
                                  int stream, int n_streams, const int32_t* __restrict__ major,
                                  const int32_t* __restrict__ minor, const int32_t* __restrict__ qslot,
                                  const int32_t* __restrict__ runs, int64_t n_events) {
  const int64_t row = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= r1) return;
  const uint64_t hi = T.hi[row];
  const uint64_t rmask = (1ull << RANK_BITS) - 1;
  if (!chunk || (hi & rmask) == 0) {
    T.chi[row] = chunk ? (uint64_t)cseq << RANK_BITS : hi & ~rmask;
    T.clo[row] = 0;
    return;
  }
  const int64_t q = T.q[row];
  const int64_t qs = q * n_streams + stream;
  const int slot = qslot[q];
  uint64_t run = 0;
  if (slot >= 0) run = (uint64_t)runs[(int64_t)slot * n_events + (T.seq[row] - first_seq)];
  else if (slot == -2) run = T.lo[2][row];  // fan-out: the key's junction-map position
  T.chi[row] = ((uint64_t)cseq << RANK_BITS) | (uint64_t)major[qs];
  T.clo[row] = (run << RANK_BITS) | (uint64_t)minor[qs];
}

__global__ void iota_kernel(int32_t* p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (int32_t)i;
}

__global__ void gather_key_kernel(const uint64_t* __restrict__ key, const int32_t* __restrict__ perm, int64_t n,
                                  uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = key[perm[i]];
}

// sorted row i <- table row perm[i]; len[n] = 0 so that an exclusive scan of n+1 gives off[n]
__global__ void gather_rows_kernel(MatchTable T, const int32_t* __restrict__ perm, int64_t n, int64_t* __restrict__ oq,
                                   int64_t* __restrict__ okey, int64_t* __restrict__ ots, int64_t* __restrict__ oseq,
                                   int64_t* __restrict__ otb, int64_t* __restrict__ olen) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    olen[n] = 0;
    return;
  }
  const int32_t p = perm[i];
  oq[i] = T.q[p];
  okey[i] = T.key[p];
  ots[i] = T.ts[p];
  oseq[i] = T.seq[p];
  // timer rows rank 0 (append_gen_kernel) and carry their tiebreak time in lo[2]
  const bool timer = (T.hi[p] & ((1ull << RANK_BITS) - 1)) == 0;
  otb[i] = timer ? (int64_t)(T.lo[2][p] ^ 0x8000000000000000ull) : INT64_MIN;
  olen[i] = T.wlen[p];
}

__global__ void gather_words_kernel(MatchTable T, const int32_t* __restrict__ perm, int64_t n,
                                    const int64_t* __restrict__ ooff, int64_t* __restrict__ owords) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t p = perm[i];
  const int64_t* s = T.words + T.woff[p];
  int64_t* d = owords + ooff[i];
  const int64_t len = T.wlen[p];
  for (int64_t k = 0; k < len; ++k) d[k] = s[k];
}

inline unsigned grid(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

}  // namespace sdh

using sdh::MatchTable;

extern "C" hipError_t sdh_append_ratchet(const int64_t* match, int blk_recs, int wide, const int32_t* blk_count,
                                         const int32_t* blk_group, const int64_t* dst_off,
                                         const sdh::RatchetGroup* groups, const int64_t* ts, int64_t seq_base,
                                         int64_t seq_ref, const int32_t* out_rank, int n_streams, int n_blocks,
                                         MatchTable T, int64_t row0, int64_t word0, hipStream_t s) {
  if (n_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::append_ratchet_kernel, dim3(n_blocks), dim3(256), 0, s, match, blk_recs, wide, blk_count,
                     blk_group, dst_off, groups, ts, seq_base, seq_ref, out_rank, n_streams, T, row0, word0);
  return hipGetLastError();
}

extern "C" hipError_t sdh_append_chain(const int64_t* src, const int64_t* seg_off, const int64_t* seg_count,
                                       const int64_t* dst_off, int rec_words, int n_items, const int32_t* qinfo,
                                       int64_t seq_ref, const int32_t* out_rank, int n_streams, MatchTable T,
                                       int64_t row0, int64_t word0, hipStream_t s) {
  if (n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::append_chain_kernel, dim3(n_items), dim3(256), 0, s, src, seg_off, seg_count, dst_off,
                     rec_words, qinfo, seq_ref, out_rank, n_streams, T, row0, word0);
  return hipGetLastError();
}

// table words per record (tw, n_rec + 1 entries) scanned in place (tw[n_rec] = the total), so the
// host can reserve the table's words before sdh_append_gen
extern "C" size_t sdh_gen_words_temp_bytes(int64_t n_rec) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n_rec + 1));
  return b + 256;
}
extern "C" hipError_t sdh_gen_words(const int64_t* out, const int64_t* rec_off, int64_t n_rec, int64_t* tw, void* temp,
                                    size_t temp_bytes, unsigned long long* n_wide, hipStream_t s) {
  if (n_rec <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(n_wide, 0, 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sdh::gen_rec_words_kernel, dim3(sdh::grid(n_rec + 1, 256)), dim3(256), 0, s, out, rec_off, n_rec, tw,
                     n_wide);
  size_t tb = temp_bytes;
  return hipcub::DeviceScan::ExclusiveSum(temp, tb, tw, tw, (int)(n_rec + 1), s);
}

extern "C" hipError_t sdh_append_gen(const int64_t* out, const int64_t* rec_off, int64_t n_rec, int64_t seq_ref,
                                     const int32_t* out_rank, const int32_t* fan_rank, int n_streams, MatchTable T,
                                     int64_t row0, int64_t word0, const int64_t* woff, const int64_t* bts,
                                     int64_t seq_base, int bstream, const int64_t* const* qkeys, hipStream_t s) {
  if (n_rec <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::append_gen_kernel, dim3(sdh::grid(n_rec, 256)), dim3(256), 0, s, out, rec_off, n_rec,
                     seq_ref, out_rank, fan_rank, n_streams, T, row0, word0, woff, bts, seq_base, bstream, qkeys);
  return hipGetLastError();
}

extern "C" hipError_t sdh_digest_ratchet(const int64_t* match, int blk_recs, int wide, const int32_t* blk_count,
                                         const int32_t* blk_group, const int32_t* blk_side,
                                         const sdh::RatchetGroup* groups, int64_t seq_base,
                                         int n_blocks, unsigned long long* acc, hipStream_t s) {
  if (n_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::digest_ratchet_kernel, dim3(n_blocks), dim3(256), 0, s, match, blk_recs, wide, blk_count,
                     blk_group, blk_side, groups, seq_base, acc);
  return hipGetLastError();
}

// device records -> compact rows: the blocks' record counts widened and scanned into row offsets
// (row_off: n_blocks + 1 int64, the total last), then one workgroup per block
__global__ void widen_counts_kernel(const int32_t* __restrict__ c, int64_t n, int64_t* __restrict__ o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) o[i] = i < n ? (int64_t)c[i] : 0;
}
extern "C" size_t sdh_ratchet_compact_temp(int64_t n_blocks) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n_blocks + 1));
  return b;
}
extern "C" hipError_t sdh_ratchet_compact(const int64_t* match, int blk_recs, int wide, const int32_t* blk_count,
                                          const int32_t* blk_group, const int32_t* blk_side,
                                          const sdh::RatchetGroup* groups, int64_t seq_base, int n_blocks,
                                          int64_t* row_off, void* temp, size_t temp_bytes, int width, int32_t* rows,
                                          hipStream_t s) {
  if (n_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(widen_counts_kernel, dim3(sdh::grid(n_blocks + 1, 256)), dim3(256), 0, s, blk_count,
                     (int64_t)n_blocks, row_off);
  size_t tb = temp_bytes;
  hipError_t r = hipcub::DeviceScan::ExclusiveSum(temp, tb, row_off, row_off, n_blocks + 1, s);
  if (r != hipSuccess) return r;
  if (rows)
    hipLaunchKernelGGL(sdh::ratchet_compact_kernel, dim3(n_blocks), dim3(256), 0, s, match, blk_recs, wide, blk_count,
                       blk_group, blk_side, groups, row_off, seq_base, width, rows);
  return hipGetLastError();
}

// the same order-independent digest over placed compact rows [row0, row0 + n) (a placed push)
__global__ __launch_bounds__(256) void digest_compact_kernel(const int32_t* __restrict__ crow, int width, int64_t row0,
                                                             int64_t n, int64_t seq_ref, unsigned long long* acc) {
  unsigned long long h = 0, c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* r = crow + (row0 + i) * width;
    const int64_t s = seq_ref + (int64_t)r[1], s1 = s - (int64_t)r[2];
    h += sdh::mix64(sdh::mix64((uint64_t)s * 0x9E3779B97F4A7C15ull ^ (uint64_t)(int64_t)r[0]) ^ (uint64_t)s1);
    ++c;
  }
  for (int o = 32; o > 0; o >>= 1) {
    h += __shfl_down(h, o);
    c += __shfl_down(c, o);
  }
  if ((threadIdx.x & 63) == 0 && c) {
    atomicAdd(&acc[0], c);
    atomicAdd(&acc[1], h);
  }
}
extern "C" hipError_t sdh_digest_compact(const int32_t* crow, int width, int64_t row0, int64_t n, int64_t seq_ref,
                                         unsigned long long* acc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(digest_compact_kernel, dim3(1024), dim3(256), 0, s, crow, width, row0, n, seq_ref, acc);
  return hipGetLastError();
}

// Direct R18 placement: scratch bytes of the scan over `cells` (event, group) counts, and the
// exclusive scan itself (in place)
extern "C" size_t sdh_place_temp_bytes(int64_t cells) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr, (int)cells);
  return b + 256;
}
extern "C" hipError_t sdh_place_scan(int32_t* cnt, int64_t cells, void* temp, size_t temp_bytes, hipStream_t s) {
  size_t tb = temp_bytes;
  return hipcub::DeviceScan::ExclusiveSum(temp, tb, cnt, cnt, (int)cells, s);
}

// the exact int64 total of the (event, cell) counts before the int32 scan: a push with 2^31 matches
// or more would wrap the scan's offsets (engine.hip then takes the table path)
__global__ __launch_bounds__(256) void place_total_kernel(const int32_t* __restrict__ cnt, int64_t cells,
                                                          unsigned long long* __restrict__ tot) {
  unsigned long long a = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += (int64_t)gridDim.x * blockDim.x)
    a += (unsigned long long)(uint32_t)cnt[i];
  for (int o = 32; o > 0; o >>= 1) a += __shfl_down(a, o);
  if ((threadIdx.x & 63) == 0 && a) atomicAdd(tot, a);
}
extern "C" hipError_t sdh_place_total(const int32_t* cnt, int64_t cells, unsigned long long* tot, hipStream_t s) {
  hipError_t e = hipMemsetAsync(tot, 0, 8, s);
  if (e != hipSuccess || cells <= 0) return e;
  const int64_t blocks = std::min<int64_t>(1024, (cells + 255) / 256);
  hipLaunchKernelGGL(place_total_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cnt, cells, tot);
  return hipGetLastError();
}

// the ABI columns of a placed window's compact rows (po_* arrays; off has rows + 1 entries)
extern "C" hipError_t sdh_compact_fill(const int32_t* crow, int width, int64_t rows, const int64_t* ts_log,
                                       int64_t seq_ref, int64_t* oq, int64_t* okey, int64_t* ots, int64_t* oseq,
                                       int64_t* otb, int64_t* ooff, int64_t* owords, hipStream_t s) {
  hipLaunchKernelGGL(sdh::compact_fill_kernel, dim3(sdh::grid(rows + 1, 256)), dim3(256), 0, s, crow, width, rows,
                     ts_log, seq_ref, oq, okey, ots, oseq, otb, ooff, owords);
  return hipGetLastError();
}

extern "C" hipError_t sdh_placed_to_table(const int32_t* crow, int width, int64_t n, const int64_t* ts_log,
                                          int64_t seq_ref, const int32_t* out_rank, const int32_t* qinfo,
                                          int n_streams, MatchTable T, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::placed_to_table_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, crow, width, n, ts_log,
                     seq_ref, out_rank, qinfo, n_streams, T);
  return hipGetLastError();
}

// the R18-sorted table rows (perm from sdh_poll_sort) as compact rows; *err (device) = 1 when some
// row does not fit the compact form
extern "C" hipError_t sdh_table_compact(MatchTable T, const int32_t* perm, int64_t n, int width, int64_t seq_ref,
                                        int32_t* crow, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::table_compact_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, T, perm, n, width, seq_ref,
                     crow, err);
  return hipGetLastError();
}

// ---- multi-GPU gather (comm.h): each sorted row's merge key ----
// The poll's sort key, most significant first: [chi, clo] when the window saw a chunk push, hi, then
// [lo2, lo1, lo0] when the program has absent states (timer rows of one seq from several ranks are
// ordered by (tb, query, key)). The words the poll did not sort on are zero in every row, and rows
// of different ranks never tie on the words used, so per-rank runs merge into the engine's order.
__device__ __forceinline__ void put_merge_key(uint64_t* w, uint64_t chi, uint64_t clo, uint64_t hi, uint64_t l2,
                                              uint64_t l1, uint64_t l0, int chunk_words, int lo_words) {
  int k = 0;
  if (chunk_words) {
    w[k++] = chi;
    w[k++] = clo;
  }
  w[k++] = hi;
  if (lo_words) {
    w[k++] = l2;
    w[k++] = l1;
    w[k++] = l0;
  }
}

__global__ __launch_bounds__(256) void merge_keys_table_kernel(MatchTable T, const int32_t* __restrict__ perm,
                                                               int64_t n, int chunk_words, int lo_words, int chunked,
                                                               uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t p = perm[i];
  const int kw = 2 * chunk_words + 1 + 3 * lo_words;
  const uint64_t hi = T.hi[p];
  const uint64_t chi = chunked ? T.chi[p] : hi & ~((1ull << sdh::RANK_BITS) - 1);
  const uint64_t clo = chunked ? T.clo[p] : 0ull;
  put_merge_key(keys + i * kw, chi, clo, hi, T.lo[2][p], T.lo[1][p], T.lo[0][p], chunk_words, lo_words);
}

// a placed window's compact rows (the keys placed_to_table_kernel would give them)
__global__ __launch_bounds__(256) void merge_keys_placed_kernel(const int32_t* __restrict__ crow, int width, int64_t n,
                                                                int64_t seq_ref, const int32_t* __restrict__ out_rank,
                                                                const int32_t* __restrict__ qinfo, int n_streams,
                                                                int chunk_words, int lo_words,
                                                                uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t* r = crow + i * width;
  const int qq = r[0];
  const int64_t e2 = seq_ref + (int64_t)r[1], e1 = e2 - (int64_t)r[2];
  const int kw = 2 * chunk_words + 1 + 3 * lo_words;
  const uint64_t hi = sdh::hi_key(e2, seq_ref, out_rank[(int64_t)qq * n_streams + qinfo[2 * qq + 1]]);
  put_merge_key(keys + i * kw, hi & ~((1ull << sdh::RANK_BITS) - 1), 0ull, hi, 0ull, 0ull, (uint64_t)e1, chunk_words,
                lo_words);
}

extern "C" hipError_t sdh_merge_keys_table(MatchTable T, const int32_t* perm, int64_t n, int chunk_words, int lo_words,
                                           int chunked, uint64_t* keys, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_keys_table_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, T, perm, n, chunk_words,
                     lo_words, chunked, keys);
  return hipGetLastError();
}

extern "C" hipError_t sdh_merge_keys_placed(const int32_t* crow, int width, int64_t n, int64_t seq_ref,
                                            const int32_t* out_rank, const int32_t* qinfo, int n_streams,
                                            int chunk_words, int lo_words, uint64_t* keys, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_keys_placed_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, crow, width, n, seq_ref,
                     out_rank, qinfo, n_streams, chunk_words, lo_words, keys);
  return hipGetLastError();
}

// ---- sdh_engine_poll_compact_ex: compact rows for every match ----
// per sorted row the chain words it needs (a slot of >= 2 events: its count, then its distances);
// cw[n] = 0 for the exclusive scan
__global__ __launch_bounds__(256) void ex_chain_words_kernel(MatchTable T, const int32_t* __restrict__ perm, int64_t n,
                                                             int64_t* __restrict__ cw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    cw[n] = 0;
    return;
  }
  const int32_t p = perm[i];
  const int64_t* w = T.words + T.woff[p];
  const int64_t len = T.wlen[p];
  int64_t t = 0;
  for (int64_t j = 0; j < len;) {
    const int64_t c = w[j];
    if (c >= 2) t += 1 + c;
    j += 1 + c;
  }
  cw[i] = t;
}

// the rows (sdh_matches_compact_ex), their chains at coff[i], keys and timer tiebreaks; err = 1 when a
// distance or a chain offset does not fit int32, or a row has more slots than the width
__global__ __launch_bounds__(256) void ex_rows_kernel(MatchTable T, const int32_t* __restrict__ perm, int64_t n,
                                                      int width, int64_t seq_ref, const int64_t* __restrict__ coff,
                                                      int32_t* __restrict__ rows, int32_t* __restrict__ chain,
                                                      int64_t* __restrict__ okey, int64_t* __restrict__ otb,
                                                      int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t p = perm[i];
  int32_t* o = rows + i * width;
  const int64_t sq = T.seq[p];
  bool bad = sq - seq_ref > INT32_MAX || sq < seq_ref;
  o[0] = (int32_t)T.q[p];
  o[1] = (int32_t)(sq - seq_ref);
  const int64_t* w = T.words + T.woff[p];
  const int64_t len = T.wlen[p];
  int64_t ref = coff[i];
  int slot = 0;
  for (int64_t j = 0; j < len && !bad; ++slot) {
    const int64_t c = w[j];
    if (2 + slot >= width) {
      bad = true;
      break;
    }
    int32_t v = INT32_MIN;
    if (c == 1) {
      const int64_t d = sq - w[j + 1];
      if (d < 0 || d > INT32_MAX) bad = true;
      v = (int32_t)d;
    } else if (c >= 2) {
      if (ref + c >= INT32_MAX) bad = true;
      chain[ref] = (int32_t)c;
      for (int64_t k = 0; k < c; ++k) {
        const int64_t d = sq - w[j + 1 + k];
        if (d < 0 || d > INT32_MAX) bad = true;
        chain[ref + 1 + k] = (int32_t)d;
      }
      v = (int32_t)(-(ref + 1));
      ref += 1 + c;
    }
    o[2 + slot] = v;
    j += 1 + c;
  }
  for (int k = 2 + slot; k < width; ++k) o[k] = INT32_MIN;
  if (okey) okey[i] = T.key[p];
  if (otb) {
    const bool timer = (T.hi[p] & ((1ull << sdh::RANK_BITS) - 1)) == 0;
    otb[i] = timer ? (int64_t)(T.lo[2][p] ^ 0x8000000000000000ull) : INT64_MIN;
  }
  if (bad) atomicOr(err, 1);
}

__global__ void fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

extern "C" size_t sdh_ex_temp_bytes(int64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n + 1));
  return b + 256;
}
// chain word offsets of the sorted rows (cw: n + 1 entries, scanned in place; cw[n] = the total)
extern "C" hipError_t sdh_ex_chain_words(MatchTable T, const int32_t* perm, int64_t n, int64_t* cw, void* temp,
                                         size_t temp_bytes, hipStream_t s) {
  hipLaunchKernelGGL(ex_chain_words_kernel, dim3(sdh::grid(n + 1, 256)), dim3(256), 0, s, T, perm, n, cw);
  size_t tb = temp_bytes;
  return hipcub::DeviceScan::ExclusiveSum(temp, tb, cw, cw, (int)(n + 1), s);
}
extern "C" hipError_t sdh_ex_rows(MatchTable T, const int32_t* perm, int64_t n, int width, int64_t seq_ref,
                                  const int64_t* coff, int32_t* rows, int32_t* chain, int64_t* okey, int64_t* otb,
                                  int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ex_rows_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, T, perm, n, width, seq_ref, coff, rows,
                     chain, okey, otb, err);
  return hipGetLastError();
}
extern "C" hipError_t sdh_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_i64_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}

// Scratch the poll needs for n rows (bytes): hipcub temp storage.
extern "C" size_t sdh_poll_temp_bytes(int64_t n) {
  size_t a = 0, b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs((void*)nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 64);
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n + 1));
  return (a > b ? a : b) + 256;
}

// R18 sort of the table's n rows and the gather of the ABI arrays except the words (device
// pointers; off has n+1 entries). n_lo tiebreak passes; lo_bits / hi_bits bound the key bits that
// vary. kbuf: 2 x n keys, pbuf: 2 x n permutation entries, olen: n + 1. On return *perm_out is the
// sorted permutation (inside pbuf) and *total_words (host) receives off[n] once the stream has run.
extern "C" hipError_t sdh_chunk_keys(MatchTable T, int64_t r0, int64_t r1, int chunk, int64_t cseq, int64_t first_seq,
                                     int stream, int n_streams, const int32_t* major, const int32_t* minor,
                                     const int32_t* qslot, const int32_t* runs, int64_t n_events, hipStream_t s) {
  if (r1 <= r0) return hipSuccess;
  hipLaunchKernelGGL(sdh::chunk_keys_kernel, dim3(sdh::grid(r1 - r0, 256)), dim3(256), 0, s, T, r0, r1, chunk, cseq,
                     first_seq, stream, n_streams, major, minor, qslot, runs, n_events);
  return hipGetLastError();
}

// clo_bits > 0: the window holds chunk rows, two more passes (clo, then chi) after hi
extern "C" hipError_t sdh_poll_sort(MatchTable T, int64_t n, int n_lo, int lo_bits, int hi_bits, int clo_bits,
                                    uint64_t* kbuf, int32_t* pbuf, void* temp, size_t temp_bytes, int64_t* oq,
                                    int64_t* okey, int64_t* ots, int64_t* oseq, int64_t* otb, int64_t* olen,
                                    int64_t* ooff, int32_t** perm_out, int64_t* total_words, hipStream_t s) {
  using namespace sdh;
  *total_words = 0;
  *perm_out = pbuf;
  if (n <= 0) return hipSuccess;
  int32_t* perm = pbuf;
  int32_t* perm2 = pbuf + n;
  uint64_t* k1 = kbuf;
  uint64_t* k2 = kbuf + n;
  hipLaunchKernelGGL(iota_kernel, dim3(grid(n, 256)), dim3(256), 0, s, perm, n);
  auto pass = [&](const uint64_t* key, int bits) -> hipError_t {
    if (bits <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_key_kernel, dim3(grid(n, 256)), dim3(256), 0, s, key, perm, n, k1);
    size_t tb = temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, tb, k1, k2, perm, perm2, (int)n, 0, bits, s);
    if (e != hipSuccess) return e;
    int32_t* t = perm;
    perm = perm2;
    perm2 = t;
    return hipGetLastError();
  };
  for (int k = 0; k < n_lo && k < MAXLO; ++k) {
    hipError_t e = pass(T.lo[k], lo_bits);
    if (e != hipSuccess) return e;
  }
  hipError_t e = pass(T.hi, hi_bits);
  if (e != hipSuccess) return e;
  if (clo_bits > 0) {
    e = pass(T.clo, clo_bits);
    if (e != hipSuccess) return e;
    e = pass(T.chi, hi_bits);
    if (e != hipSuccess) return e;
  }
  *perm_out = perm;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid(n + 1, 256)), dim3(256), 0, s, T, perm, n, oq, okey, ots, oseq, otb,
                     olen);
  size_t tb = temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(temp, tb, olen, ooff, (int)(n + 1), s);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(total_words, ooff + n, 8, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

// the words of the sorted rows (owords holds off[n] entries)
extern "C" hipError_t sdh_poll_words(MatchTable T, const int32_t* perm, int64_t n, const int64_t* ooff,
                                     int64_t* owords, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::gather_words_kernel, dim3(sdh::grid(n, 256)), dim3(256), 0, s, T, perm, n, ooff, owords);
  return hipGetLastError();
}
