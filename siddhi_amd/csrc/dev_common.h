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

// The logical item of this workgroup. Observed dispatch deals workgroups round-robin over the 8
// XCDs, blocks b and b + 8 sharing one (MI355X_MICROARCH.md; speed only, never correctness). With
// `xcd` set the launch pads its grid to a multiple of 8 and each XCD takes one contiguous range of
// items, so neighbouring items -- one key's groups, one event chunk's groups -- read the inputs they
// share (the key's events, a tile, directory lines) through one XCD's L2 instead of all eight.
// Items at or past the launch's count return.
__device__ __forceinline__ int64_t grid_item(int xcd) {
  const int64_t b = blockIdx.x;
  if (!xcd) return b;
  return (b & 7) * (int64_t)(gridDim.x >> 3) + (b >> 3);
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
// Device records (write_records == 2, SDH_FLAG_DEVICE_MATCHES): the records stay in the buffer for a
// consumer (sdh_engine_poll_records walks them by their first word's length; include/siddhi_hip.h) and
// no record index is kept. In normal mode each record's offset is also listed in rec_off (the device
// match table finds records by it, matches.hip); a record fits only if its words and its index entry
// both do. Either way a reservation past the buffer sets `over`, and the host grows the buffer and
// re-runs the push exactly.
// A pad record (device records: the unused tail of a wave's reserved run, WaveOutT) has first word
// (uint32)(-(REC_PAD + words)): it spans `words` words, of which only the first is written.
constexpr int REC_PAD = 4 << 16;
struct LaneOut {
  int64_t* out;
  int64_t cap;
  unsigned long long* next;
  bool ring;  // device records
  int64_t* rec_off;
  int64_t rec_cap;
  unsigned long long* rec_next;
  bool over = false;
  __device__ void close() {}
  // nl records of `words` words each, contiguous
  __device__ int64_t* reserve_n(int nl, int words) {
    const int64_t tw = (int64_t)nl * words;
    const unsigned long long o = atomicAdd(next, (unsigned long long)tw);
    if ((int64_t)(o + tw) > cap) {
      over = true;
      return nullptr;
    }
    if (ring) return out + o;
    const unsigned long long r = atomicAdd(rec_next, (unsigned long long)nl);
    if ((int64_t)(r + nl) > rec_cap) {
      over = true;
      return nullptr;
    }
    for (int i = 0; i < nl; ++i) rec_off[r + i] = (int64_t)o + (int64_t)i * words;
    return out + o;
  }
  __device__ int64_t* reserve(int words) {
    const unsigned long long o = atomicAdd(next, (unsigned long long)words);
    if ((int64_t)(o + words) > cap) {
      over = true;
      return nullptr;
    }
    if (ring) return out + o;
    const unsigned long long r = atomicAdd(rec_next, 1ull);
    if ((int64_t)r >= rec_cap) {
      over = true;
      return nullptr;
    }
    rec_off[r] = (int64_t)o;
    return out + o;
  }
  // device records: the words [o, o + words) hold no record
  __device__ void pad(int64_t o, int64_t words) {
    if (words > 0 && o < cap) out[o] = (int64_t)(uint64_t)(uint32_t)(-(REC_PAD + (int32_t)words));
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
// CAPW_: words in the LDS buffer. Every flush takes two atomics on the chip-wide counters, which
// serialise once the match rate is high (C3: 512 words -> 42 ms/step, 1536 -> 24), while a larger
// buffer costs resident waves (4096 -> 38 ms); K_part uses 1536, K_seq 1024 (measured)
// Device records (SDH_FLAG_DEVICE_MATCHES) reserve SDH_RING_CHUNK buffers' worth of the buffer per
// atomic: the flush's round trip on the chip-wide counter stalls the whole wave (C3 chunk 1: 23.4
// ms/step, 4: 20.7, 16: 20.7; C4 27.3 / 25.9 / 26.1). The unused tail of a run becomes a pad record.
// CHUNK 1 (K_slab: a wave flushes about once, a few records) reserves exactly what each flush needs.
#ifndef SDH_RING_CHUNK
#define SDH_RING_CHUNK 4
#endif
template <int CAPW_, bool SWZ = false, int CHUNK = SDH_RING_CHUNK>
struct WaveOutT {
  static constexpr int CAPW = CAPW_;
  static constexpr int CAPR = CAPW / NREC_MIN_WORDS + 1;  // records (>= 3 words each: the narrow ones)
  static constexpr int RBITS = CAPR < 1024 ? 10 : 11;       // bits of a record count <= CAPR
  // SWZ: LDS word x of the buffer lives at x ^ ((x >> 4) & 15) (an XOR swizzle inside each 16-word
  // block). The lanes of one collective emit write records of `words` words at lane-strided offsets,
  // and a ds_write_b64 serves 16 contiguous lanes per cycle on 16 qword banks, so K_part's 4- and
  // 8-word records would put 4 or 8 lanes on one bank; the swizzle spreads them (a 16-word block's
  // lanes get distinct banks for any power-of-two stride: C3 9.6 % -> 1.3 % of LDS cycles). Odd
  // record lengths (K_seq's 13 words) are conflict-free unswizzled and keep the plain layout (the
  // swizzle put C4 at 5.0 % from 0.6 %).
  static_assert(!SWZ || CAPW % 16 == 0, "the LDS swizzle works in 16-word blocks");
  static constexpr int PADW = CAPW;
  __device__ static int pidx(int x) { return SWZ ? x ^ ((x >> 4) & 15) : x; }
  struct Rec {  // a record's words in the padded buffer (pointer-like: r[i], r + k)
    int64_t* b;
    int off;
    __device__ int64_t& operator[](int i) const { return b[pidx(off + i)]; }
    __device__ Rec operator+(int d) const { return Rec{b, off + d}; }
  };
  struct Shared {
    int64_t buf[PADW];
    int32_t roff[CAPR];
    int64_t base, rbase;
    int32_t used, nrec;
    int64_t cbase, cleft;  // device records: the wave's reserved run of the buffer (SDH_RING_CHUNK)
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
  // ordering of the wave's own LDS accesses across lanes. The work group is one wave and a wave's
  // LDS operations complete in issue order, so only the compiler must not move them (a wavefront-
  // scope fence emits no wait)
  __device__ static void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
  __device__ static unsigned long long active() { return __ballot(1); }
  __device__ static unsigned long long below() { return (1ull << __lane_id()) - 1ull; }
  __device__ void init() {
    if (__lane_id() == 0) {
      st(sh->used, 0);
      st(sh->nrec, 0);
      st(sh->cleft, (int64_t)0);
    }
    wave_fence();
  }
  // copy the buffer out (active lanes cooperate)
  __device__ void flush() {
    wave_fence();  // the records' LDS words are written
    const unsigned long long m = active();
    const int cnt = __popcll(m), me = __popcll(m & below()), lead = __ffsll((long long)m) - 1;
    const int n = ld(sh->used), nr = ld(sh->nrec);
    if (n == 0) return;
    if (__lane_id() == lead) {
      // device records: one reservation per CHUNK buffers' worth of words (a run's unused tail
      // becomes a pad record)
      unsigned long long o;
      if (CHUNK > 1 && g.ring) {
        if (ld(sh->cleft) < n) {
          g.pad(ld(sh->cbase), ld(sh->cleft));
          st(sh->cbase, (int64_t)atomicAdd(g.next, (unsigned long long)(CHUNK * CAPW)));
          st(sh->cleft, (int64_t)(CHUNK * CAPW));
        }
        o = (unsigned long long)ld(sh->cbase);
        st(sh->cbase, ld(sh->cbase) + n);
        st(sh->cleft, ld(sh->cleft) - n);
      } else {
        o = atomicAdd(g.next, (unsigned long long)n);
      }
      int64_t base = (int64_t)o, rbase = 0;
      if ((int64_t)(o + n) > g.cap) base = -1;
      if (!g.ring) {
        const unsigned long long r = atomicAdd(g.rec_next, (unsigned long long)nr);
        if ((int64_t)(r + nr) > g.rec_cap) base = -1;
        rbase = (int64_t)r;
      }
      st(sh->base, base);
      st(sh->rbase, rbase);
    }
    wave_fence();
    const int64_t base = ld(sh->base), rbase = ld(sh->rbase);
    if (base < 0) {
      g.over = true;
    } else if (g.ring) {
      for (int i = me; i < n; i += cnt) g.out[base + i] = sh->buf[pidx(i)];
    } else {
      for (int i = me; i < n; i += cnt) g.out[base + i] = sh->buf[pidx(i)];
      for (int i = me; i < nr; i += cnt) g.rec_off[rbase + i] = base + sh->roff[i];
    }
    wave_fence();
    if (__lane_id() == lead) {  // (one lane: 64 same-address writes serialise as bank conflicts)
      st(sh->used, 0);
      st(sh->nrec, 0);
    }
    wave_fence();
  }
  // `nl` records of `words` words each for this lane (collective over the active lanes: they all
  // call it at the same point), written by fill(r) (r: a Rec into the LDS buffer, or an int64_t* into
  // a global reservation; generic callbacks index both alike): record i at r + i * words, into the LDS
  // buffer. A call larger than the buffer's free room goes in rounds: each round places the lanes
  // (in lane order) whose words and records fit, then the buffer is flushed. Only a lane whose own
  // records exceed the whole buffer reserves globally, as LaneOut does.
  // uw: every lane's records have the same, wave-uniform, word count (the word prefixes are then the
  // record prefixes times it: rbits ballots -- nl < 2^rbits -- instead of 23)
  template <class F>
  __device__ void emit_n(int nl, int words, F&& fill, bool uw = false, int rbits = RBITS) {
    const unsigned long long lt = below();
    const bool big = nl * words > CAPW || nl > CAPR;
    const int mtw = big ? 0 : nl * words, mnl = big ? 0 : nl;
    int wpre = 0, wtot = 0, rpre = 0;  // exclusive lane prefixes, total words (ballot bits)
    if (uw) {
      int rtot = 0;
#pragma unroll
      for (int b = 0; b < RBITS; ++b) {  // mnl <= CAPR
        if (b >= rbits) break;
        const unsigned long long mb = __ballot((mnl >> b) & 1);
        rpre += __popcll(mb & lt) << b;
        rtot += __popcll(mb) << b;
      }
      wpre = rpre * words;
      wtot = rtot * words;
    } else {
#pragma unroll
      for (int b = 0; b < 13; ++b) {  // mtw <= CAPW
        const unsigned long long mb = __ballot((mtw >> b) & 1);
        wpre += __popcll(mb & lt) << b;
        wtot += __popcll(mb) << b;
      }
#pragma unroll
      for (int b = 0; b < RBITS; ++b) {  // mnl <= CAPR
        const unsigned long long mb = __ballot((mnl >> b) & 1);
        rpre += __popcll(mb & lt) << b;
      }
    }
    place(nl, words, big, mtw, mnl, wpre, wtot, rpre, fill);
  }
  // one record of `words` (wave-uniform) words per active lane: the prefixes are mbcnt
  template <class F>
  __device__ void emit_u(int words, F&& fill) {
    const unsigned long long act = active();
    const bool big = words > CAPW;
    const int me = __popcll(act & below()), n = __popcll(act);
    place(1, words, big, big ? 0 : words, big ? 0 : 1, big ? 0 : me * words, big ? 0 : n * words, big ? 0 : me,
          fill);
  }
  // the placement rounds of a call (see emit_n)
  template <class F>
  __device__ void place(int nl, int words, bool big, int mtw, int mnl, int wpre, int wtot, int rpre, F&& fill) {
    int wdone = 0, rdone = 0;  // (uniform) words / records of this call placed so far
    while (wdone < wtot) {
      const int used = ld(sh->used), nr = ld(sh->nrec);
      const bool fits = mnl > 0 && wpre >= wdone && wpre + mtw - wdone <= CAPW - used &&
                        rpre + mnl - rdone <= CAPR - nr;
      const unsigned long long fm = __ballot(fits);
      if (!fm) {  // not even the first pending lane fits: empty the buffer
        flush();
        continue;
      }
      // the fitting lanes are a prefix of the pending ones (the prefix sums are monotone)
      const int hi = 63 - __builtin_clzll(fm);
      const int wend = __builtin_amdgcn_readlane(wpre + mtw, hi), rend = __builtin_amdgcn_readlane(rpre + mnl, hi);
      const int off = used + wpre - wdone, r0 = nr + rpre - rdone;
      if (fits)
        for (int i = 0; i < mnl; ++i) sh->roff[r0 + i] = off + i * words;
      wave_fence();
      if (__lane_id() == __ffsll((long long)active()) - 1) {  // (one lane, as in flush)
        st(sh->used, used + wend - wdone);
        st(sh->nrec, nr + rend - rdone);
      }
      wave_fence();
      if (fits) fill(Rec{sh->buf, off});
      wdone = wend;
      rdone = rend;
    }
    if (big) {
      int64_t* r = g.reserve_n(nl, words);
      if (r) fill(r);
    }
  }
  // this lane's record of `words` words, written by fill(r)
  template <class F>
  __device__ void emit(int words, F&& fill) {
    emit_n(1, words, fill);
  }
  __device__ void close() {
    flush();
    if (CHUNK > 1) {
      if (g.ring && __lane_id() == __ffsll((long long)active()) - 1) g.pad(ld(sh->cbase), ld(sh->cleft));
      wave_fence();
    }
    over |= g.over;
  }
};
using WaveOut = WaveOutT<1536, true>;  // K_part
using SeqWaveOut = WaveOutT<1024>; // K_seq

__device__ __forceinline__ bool expired(int64_t ts1, int64_t ts, int64_t within) {
  if (within < 0) return false;
  const int64_t d = (int64_t)((uint64_t)ts1 - (uint64_t)ts);
  const int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
  return a > within;
}

}  // namespace dev
}  // namespace sdh
