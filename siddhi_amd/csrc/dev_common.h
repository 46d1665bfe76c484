// dev_common.h -- device helpers shared by the NFA kernels (nfa_gen.hip, nfa_part.hip) and by the
// shape-compiled kernels built at engine creation (spec.hip: seq_body.h / part_body.h compiled at
// run time with hiprtc, so this header also builds without the host's system headers).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "kgen.h"
#include "nfa_types.h"

namespace sdh {
namespace dev {

template <class T, int N>
__device__ __forceinline__ T gpick(const T (&arr)[N], int idx) {
  T v = arr[0];
#pragma unroll
  for (int c = 1; c < N; ++c) v = (idx == c) ? arr[c] : v;
  return v;
}

// attribute word `attr` of batch event e: int / string id sign-extended, float bits, long / double
// bits, bool byte; *isnull from the column's null bytes
__device__ __forceinline__ int64_t raw_word(const StreamBatch& b, int attr, int64_t e, bool& isnull) {
  const void* p = gpick(b.col, attr);
  const uint8_t* nl = gpick(b.nul, attr);
  const int w = gpick(b.width, attr);
  isnull = nl && nl[e];
  if (w == 8) return ((const int64_t*)p)[e];
  if (w == 4) return (int64_t)((const int32_t*)p)[e];
  return (int64_t)((const uint8_t*)p)[e];
}

// match output: one flat word buffer; each record is reserved with an atomic add of its length
// (the backend's atomic optimizer folds a wave's same-address adds into one atomic + a scan).
// Ring mode (write_records == 2, SDH_FLAG_DEVICE_MATCHES): every record is still written, at its
// offset modulo the buffer less a one-record margin, because nobody reads it back. In normal mode
// each record's offset is also listed in rec_off (the device match table finds records by it,
// matches.hip); a record fits only if its words and its index entry both do.
struct LaneOut {
  int64_t* out;
  int64_t cap;
  unsigned long long* next;
  bool ring;
  int64_t* rec_off;
  int64_t rec_cap;
  unsigned long long* rec_next;
  bool over = false;
  __device__ void close() {}
  __device__ int64_t* reserve(int words) {
    const unsigned long long o = atomicAdd(next, (unsigned long long)words);
    if (ring) return out + (int64_t)(o % (unsigned long long)(cap - GEN_RING_MARGIN));
    if ((int64_t)(o + words) > cap) {
      over = true;
      return nullptr;
    }
    const unsigned long long r = atomicAdd(rec_next, 1ull);
    if ((int64_t)r >= rec_cap) {
      over = true;
      return nullptr;
    }
    rec_off[r] = (int64_t)o;
    return out + o;
  }
};

// Wave-buffered match output: a work group is ONE wave; its records are assembled in an LDS buffer
// and flushed to the global buffer with one word reservation and one record-index reservation per
// flush (a per-record atomic on the two global counters serialises the whole chip once the match
// rate is ~1e9/s). Collective over the lanes active at the call: every active lane calls reserve()
// (its record's words) at the same point. A lane's offset is the sum of the active lanes below it,
// computed from six ballots of the record lengths' bits (no LDS atomics: the backend lowers a
// divergent atomic add into a loop over the active lanes). Records of one call land in lane order;
// the device match table orders rows by their keys anyway (R18). A call whose records cannot fit an
// empty buffer reserves globally per lane, as LaneOut does.
struct WaveOut {
  static constexpr int CAPW = 512;             // words in the LDS buffer (4 KiB: occupancy)
  static constexpr int CAPR = CAPW / 7 + 1;    // records (>= 7 words each)
  struct Shared {
    int64_t buf[CAPW];
    int32_t roff[CAPR];
    int64_t base, rbase;
    int32_t used, nrec;
  };
  // the wave's shared counters: relaxed atomics, so no lane keeps a stale copy in a register (other
  // lanes update them) and, unlike volatile, the accesses stay ds_ operations
  template <class T>
  __device__ static T ld(T& x) { return __hip_atomic_load(&x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
  template <class T>
  __device__ static void st(T& x, T v) { __hip_atomic_store(&x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
  LaneOut g;
  Shared* sh;
  bool over = false;
  __device__ static unsigned long long active() { return __ballot(1); }
  __device__ static unsigned long long below() { return (1ull << __lane_id()) - 1ull; }
  __device__ void init() {
    if (__lane_id() == 0) {
      st(sh->used, 0);
      st(sh->nrec, 0);
    }
    __threadfence_block();
  }
  // copy the buffer out (active lanes cooperate)
  __device__ void flush() {
    __threadfence_block();  // the records' LDS words are written
    const unsigned long long m = active();
    const int cnt = __popcll(m), me = __popcll(m & below()), lead = __ffsll((long long)m) - 1;
    const int n = ld(sh->used), nr = ld(sh->nrec);
    if (n == 0) return;
    if (__lane_id() == lead) {
      const unsigned long long o = atomicAdd(g.next, (unsigned long long)n);
      int64_t base = (int64_t)o, rbase = 0;
      if (!g.ring) {
        if ((int64_t)(o + n) > g.cap) base = -1;
        const unsigned long long r = atomicAdd(g.rec_next, (unsigned long long)nr);
        if ((int64_t)(r + nr) > g.rec_cap) base = -1;
        rbase = (int64_t)r;
      }
      st(sh->base, base);
      st(sh->rbase, rbase);
    }
    __threadfence_block();
    const int64_t base = ld(sh->base), rbase = ld(sh->rbase);
    if (base < 0) {
      g.over = true;
    } else if (g.ring) {
      const int64_t rc = g.cap - GEN_RING_MARGIN, b0 = (int64_t)((unsigned long long)base % (unsigned long long)rc);
      for (int i = me; i < n; i += cnt) g.out[b0 + i < rc ? b0 + i : b0 + i - rc] = sh->buf[i];
    } else {
      for (int i = me; i < n; i += cnt) g.out[base + i] = sh->buf[i];
      for (int i = me; i < nr; i += cnt) g.rec_off[rbase + i] = base + sh->roff[i];
    }
    __threadfence_block();
    st(sh->used, 0);  // (every active lane writes the same values)
    st(sh->nrec, 0);
    __threadfence_block();
  }
  // this lane's record of `words` words, written by fill(int64_t* r): into the LDS buffer, or for
  // an oversized call straight into the global buffer (two instantiations, so the LDS stores are
  // ds_ writes, not flat ones); skipped once the global buffer overflowed
  template <class F>
  __device__ void emit(int words, F&& fill) {
    const unsigned long long m = active(), lt = below();
    const int cnt = __popcll(m), rank = __popcll(m & lt);
    int prefix = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const unsigned long long mb = __ballot((words >> b) & 1);
      prefix += __popcll(mb & lt) << b;
      total += __popcll(mb) << b;
    }
    if (__ballot(words >= 64) || total > CAPW || cnt > CAPR) {  // (uniform)
      int64_t* r = g.reserve(words);
      if (r) fill(r);
      return;
    }
    if (ld(sh->used) + total > CAPW || ld(sh->nrec) + cnt > CAPR) flush();
    const int base = ld(sh->used), nr = ld(sh->nrec);
    const int off = base + prefix;
    sh->roff[nr + rank] = off;
    __threadfence_block();
    st(sh->used, base + total);  // (every active lane writes the same values)
    st(sh->nrec, nr + cnt);
    fill(sh->buf + off);
  }
  // room for this lane's record of `words` words: a pointer into the LDS buffer (or, for an
  // oversized call, into the global buffer); nullptr once the global buffer overflowed
  __device__ int64_t* reserve(int words) {
    const unsigned long long m = active(), lt = below();
    const int cnt = __popcll(m), rank = __popcll(m & lt);
    int prefix = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const unsigned long long mb = __ballot((words >> b) & 1);
      prefix += __popcll(mb & lt) << b;
      total += __popcll(mb) << b;
    }
    if (__ballot(words >= 64) || total > CAPW || cnt > CAPR) return g.reserve(words);  // (uniform)
    if (ld(sh->used) + total > CAPW || ld(sh->nrec) + cnt > CAPR) flush();
    const int base = ld(sh->used), nr = ld(sh->nrec);
    const int off = base + prefix;
    sh->roff[nr + rank] = off;
    __threadfence_block();
    st(sh->used, base + total);  // (every active lane writes the same values)
    st(sh->nrec, nr + cnt);
    return sh->buf + off;
  }
  __device__ void close() {
    flush();
    over |= g.over;
  }
};

__device__ __forceinline__ bool expired(int64_t ts1, int64_t ts, int64_t within) {
  if (within < 0) return false;
  const int64_t d = (int64_t)((uint64_t)ts1 - (uint64_t)ts);
  const int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
  return a > within;
}

}  // namespace dev
}  // namespace sdh
