// nfa_slab.hip -- K_slab: distinct-stream patterns on sparse per-partial entries (slab.h: shapes and
// the exactness argument), the C5 family at config scale (100K patterns x 1M partition keys).
//
// State. Only partials that exist are stored. The entries of the 64 instances (query, key) of one
// wave -- a group of 64 same-shape queries for one key -- form a BLOCK, sorted by lane, in a slab
// of sub-rings in HBM; a dense directory [key][group] holds each block's (offset, entries, states
// with a non-empty list). An instance holding only its armed start state has no entry: PartitionRuntime
// clones a key's runtime lazily (PartitionRuntime.java:257-306) and a fresh clone holds nothing but
// the seed (StreamPreStateProcessor.init:157-166), so an absent entry IS that state.
//
// Mapping to CDNA4: item = (one key's events of the pushed stream, one group); one wave per item.
// The pushed stream feeds one state of every query of the group's shape (slab.h), so an item whose
// block has an empty list for that state costs one directory read. Otherwise the wave copies its
// block into LDS (coalesced), stages the key's events 64 at a time in LDS (read by broadcast), and
// each lane steps its own entries; matches go out through the wave-buffered LDS record buffer
// (dev::WaveOutT). The changed block is written to a NEW place (sub-ring bump allocation, one atomic
// per item), the directory entry is replaced and the old value journaled: a failed push (LDS
// capacity, slab space, output overflow) is undone by restoring the journal, and re-run exactly.
// Garbage (superseded blocks) is reclaimed between pushes by moving the live blocks of a sub-ring's
// oldest half to its head (slab_move_kernel), or by moving everything into a larger slab.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cstdlib>

#include "knobs.h"
#include "dev_common.h"
#include "slab.h"

namespace sdh {

// (C5 emits ~0.6 records per work item: a small output buffer leaves LDS for resident waves, and
// device records take exact reservations -- a 4-buffer chunk per emitting wave left ~490 B of pad
// per C5 match in the flat record buffer)
using SlabWaveOut = dev::WaveOutT<256, false, 1>;

namespace {

__device__ __forceinline__ uint32_t sub_of(uint64_t dir_idx, int nsub) {
  const uint32_t h = (uint32_t)((dir_idx * 0x9E3779B97F4A7C15ull) >> 32);
  return (nsub & (nsub - 1)) == 0 ? h & (uint32_t)(nsub - 1) : h % (uint32_t)nsub;  // (the same value)
}

// words [o, o + words) of sub-ring `sub` (o: offset in its buffer), or -1 when the ring is full (a
// block never wraps: an allocation that would straddle the ring's end is wasted and taken again)
__device__ __forceinline__ int64_t ring_alloc(unsigned long long* head, uint64_t tail, int64_t cap, uint32_t sub,
                                              int64_t words) {
  unsigned long long o = atomicAdd(&head[sub], (unsigned long long)words);
  if ((int64_t)(o % (unsigned long long)cap) + words > cap) o = atomicAdd(&head[sub], (unsigned long long)words);
  if ((int64_t)(o + words - tail) > cap || (int64_t)(o % (unsigned long long)cap) + words > cap) return -1;
  return (int64_t)(o % (unsigned long long)cap);
}

__device__ __forceinline__ int wave_prefix(int v, int bits, int* total) {
  const unsigned long long lt = (1ull << __lane_id()) - 1ull;
  int pre = 0, tot = 0;
  for (int b = 0; b < bits; ++b) {
    const unsigned long long m = __ballot((v >> b) & 1);
    pre += __popcll(m & lt) << b;
    tot += __popcll(m) << b;
  }
  *total = tot;
  return pre;
}

}  // namespace

// NAX: the captured words the event staging holds (the launch's widest shape); LDS bounds the resident
// waves of this kernel
template <int NAX, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void nfa_slab_kernel(SlabLaunch L) {
  using namespace slab;
  const int lane = threadIdx.x;
  const int gi = (int)dev::grid_item(L.xcd);
  if (gi >= L.n_items) return;
  const int item = L.item_list ? L.item_list[gi] : gi;
  const int seg = item / L.n_glist, g = L.glist[item % L.n_glist];
  const uint32_t kid = L.seg_kid[seg];
  if (kid == 0xFFFFFFFFu) return;  // null / foreign partition keys
  const Shape& sh = L.shapes[L.group_shape[g]];  // wave-uniform
  const int stream = L.b.stream;
  const int st = sh.proc[stream];
  const uint64_t dir_idx = (uint64_t)kid * (uint64_t)L.groups + (uint64_t)g;
  const uint64_t d0 = L.dir[dir_idx];
  const int n_old = (int)((d0 >> 40) & 0xffff);
  const uint32_t lists = (uint32_t)(d0 >> 56);
  if (st > 0 && !((lists >> st) & 1u)) return;  // no partial waits in this state's list
  const int qi = L.lane_q[(int64_t)(L.group_base + g) * 64 + lane];
  const bool live = qi >= 0;
  const kg::GQuery* __restrict__ q = L.queries + L.group_tmpl[L.group_base + g];
  // the lane's query id, `within` and filter constants: one coalesced row per value of the group's
  // lane-constant table (a lane reading its own GQuery instead touched 64 scattered lines per value)
  const kg::LaneConsts lk{nullptr, L.lconst + ((int64_t)(L.group_base + g) * L.lc_slots) * 64 + lane};
  const int EW = sh.EW;
  const int64_t e0 = L.seg_begin[seg], e1 = e0 + L.seg_len[seg];
  const int ncap = q->n_cap[stream];

  extern __shared__ uint32_t slab_lds[];  // [lcap][EW] entries: the old block, then new partials
  __shared__ int64_t t_ts[64], t_seq[64], t_w[NAX][64];
  __shared__ uint32_t t_nul[64];
  __shared__ SlabWaveOut::Shared out_sh;
  __shared__ int64_t sh_base;
  uint32_t* ent = slab_lds;
  const int cap_ent = L.lds_words / EW;  // entries this shape's rows fit in the launch's LDS
  // a block that outgrows this launch's rows: deferred to the large-LDS launch (two tiers keep most
  // waves small, so more of them are resident), or, in that launch, the push re-runs with more LDS.
  // A deferred item has changed nothing (an e1 item that grows emits nothing before its write-back)
  auto outgrown = [&]() {
    if (lane != 0) return;
    if (L.defer_cap > 0) {
      const int d = atomicAdd(L.defer_n, 1);
      if (d < L.defer_cap) {
        L.defer[d] = item;
        return;
      }
    }
    atomicOr(&L.err[0], 1);
  };
  if (n_old > cap_ent) {
    outgrown();
    return;
  }
  // the old block -> LDS (coalesced), then each lane's range (entries are sorted by lane)
  const uint32_t sub = sub_of(dir_idx, L.nsub);
  const uint32_t* old_blk = L.ring[sub] + (int64_t)(d0 & 0xffffffffull) * 4;
  for (int w = lane; w < n_old * EW; w += 64) ent[w] = old_blk[w];
  __syncthreads();
  int b_l = 0, e_l = 0;
  {
    int lo = 0, hi = n_old;  // first entry with lane >= this lane
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((int)(ent[m * EW] & EF_LANE) < lane) lo = m + 1;
      else hi = m;
    }
    b_l = lo;
    hi = n_old;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((int)(ent[m * EW] & EF_LANE) <= lane) lo = m + 1;
      else hi = m;
    }
    e_l = lo;
  }
  SlabWaveOut o;
  o.g = dev::LaneOut{L.out, L.out_cap, L.out_next, L.write_records == 2, L.rec_off, L.rec_cap, L.rec_next};
  o.sh = &out_sh;
  o.init();
  const int64_t within = lk.within();
  const int64_t qid = lk.qid();
  const int64_t key = L.key_of_id[kid];
  unsigned long long nrec = 0;
  bool changed = false, lds_over = false;
  int n_new = 0;  // wave-uniform: new entries appended after the old block
  // e1: armed unless a non-`every` start has fired (marker); new partials' position in element 1
  bool armed = live && sh.every;
  uint32_t pos1 = 0;
  if (st == 0 && live) {
    bool marker = false;
    uint32_t mx = 0;
    bool any = false;
    for (int k = b_l; k < e_l; ++k) {
      const uint32_t* e = ent + k * EW;
      if (e[0] & EF_MARKER) marker = true;
      bool in1 = false;
      for (int x = 0; x < 2; ++x)
        if (sh.nxt[0][x] >= 0 && (e[0] & in_bit(sh.nxt[0][x]))) in1 = true;
      if (in1) {
        const uint32_t p = pos_of(e, 1);
        mx = (!any || p > mx) ? p : mx;
        any = true;
      }
    }
    armed = sh.every || !marker;
    pos1 = any ? mx + 1 : 0;
  }

  for (int64_t t0 = e0; t0 < e1 && !lds_over; t0 += 64) {
    const int cnt = e1 - t0 < 64 ? (int)(e1 - t0) : 64;
    if (lane < cnt) {
      const int64_t ev = L.ev_idx[t0 + lane];
      t_ts[lane] = L.b.ts[ev];
      t_seq[lane] = L.b.seq_base + ev;
      uint32_t nb = 0;
      for (int j = 0; j < ncap; ++j) {
        bool nl = false;
        if (j < NAX) t_w[j][lane] = dev::raw_word(L.b, q->cap_attr[stream][j], ev, nl);
        if (nl) nb |= 1u << j;
      }
      t_nul[lane] = nb;
    }
    __syncthreads();
    for (int te = 0; te < cnt; ++te) {
      const Ev ev{t_ts[te], t_seq[te], &t_w[0][te], 64, t_nul[te]};
      if (st == 0) {  // e1: every passing lane opens a partial (and a non-every start disarms)
        const bool pass = armed && start_pass(sh, q, lk, ev);
        const int need = pass ? (sh.every ? 1 : 2) : 0;
        int tot = 0;
        const int pre = wave_prefix(need, 2, &tot);
        if (tot == 0) continue;
        if (n_old + n_new + tot > cap_ent) {
          lds_over = true;
          break;
        }
        if (pass) {
          uint32_t* e = ent + (n_old + n_new + pre) * EW;
          open_partial(sh, e, lane, pos1++, ev);
          if (!sh.every) {
            uint32_t* m = e + EW;
            for (int w = 0; w < EW; ++w) m[w] = 0;
            m[0] = (uint32_t)lane | EF_MARKER;
            armed = false;
          }
        }
        n_new += tot;
        changed = true;
        continue;
      }
      // a list event: each entry in the state's list steps on its own (slab.h step)
      bool moved = false;
      for (int k = b_l; k < e_l; ++k) {
        uint32_t* e = ent + k * EW;
        const int r = step(sh, q, lk, st, e, ev, within);
        changed |= r != 0;
        const bool em = (r & R_EMIT) != 0;
        if (em) ++nrec;
        if (L.write_records && __ballot(em) != 0) {  // (the collective emit only when a lane emits)
          const int words = em ? record_words(sh, e, st) : 0;
          const int64_t idx = (int64_t)pos_of(e, sh.elem[st]);
          o.emit_n(em ? 1 : 0, words, [&](auto rr) {
            write_record(sh, e, st, words, qid, key, idx, stream, ev, rr);
          });
        }
        if (r & R_MOVE) {
          e[0] |= EF_MOVED;
          moved = true;
        }
      }
      if (moved) {
        // arrivals in the next element, in the order of the list they leave (its positions): after
        // every partial already there (StreamPreStateProcessor.addState appends to newAndEvery)
        const int ne = sh.elem[st] + 1, es = sh.elem[st];
        const int n0 = sh.nxt[st][0], n1 = sh.nxt[st][1];
        uint32_t mx = 0;
        bool any = false;
        for (int k = b_l; k < e_l; ++k) {
          const uint32_t* e = ent + k * EW;
          if ((e[0] & EF_MOVED) || !((e[0] & in_bit(n0)) || (n1 >= 0 && (e[0] & in_bit(n1))))) continue;
          const uint32_t p = pos_of(e, ne);
          mx = (!any || p > mx) ? p : mx;
          any = true;
        }
        const uint32_t base = any ? mx + 1 : 0;
        for (int k = b_l; k < e_l; ++k) {
          uint32_t* e = ent + k * EW;
          if (!(e[0] & EF_MOVED)) continue;
          const uint32_t p = pos_of(e, es);
          uint32_t rank = 0;
          for (int k2 = b_l; k2 < e_l; ++k2) {
            const uint32_t* e2 = ent + k2 * EW;
            if ((e2[0] & EF_MOVED) && pos_of(e2, es) < p) ++rank;
          }
          set_pos(e, ne, base + rank);
          e[0] |= in_bit(n0) | (n1 >= 0 ? in_bit(n1) : 0u);
        }
        for (int k = b_l; k < e_l; ++k) ent[k * EW] &= ~EF_MOVED;
      }
    }
    __syncthreads();  // the tile is rewritten next
  }
  o.close();
  if (lds_over) {  // only e1 items grow (they emit nothing)
    outgrown();
    return;
  }
  if (lane == 0 && n_old) atomicAdd(&L.traffic[item & 255], (unsigned long long)n_old * EW * 4);
  if (nrec) atomicAdd(L.rec_count, nrec);
  if (o.over) atomicOr(&L.err[2], 1);
  if (!__ballot(changed)) return;
  // write-back: the lane's surviving entries (old ones still in a list, markers) then its new ones
  int m_l = 0, parts_old = 0, parts_new = 0;
  uint32_t lbits = 0;
  for (int k = b_l; k < e_l; ++k) {
    const uint32_t f = ent[k * EW];
    if (!(f & EF_MARKER)) ++parts_old;
    if ((f & EF_INLIST) || (f & EF_MARKER)) {
      ++m_l;
      lbits |= f;
      if (!(f & EF_MARKER)) ++parts_new;
    }
  }
  for (int k = n_old; k < n_old + n_new; ++k) {
    const uint32_t f = ent[k * EW];
    if ((int)(f & EF_LANE) != lane) continue;
    ++m_l;
    lbits |= f;
    if (!(f & EF_MARKER)) ++parts_new;
  }
  int M = 0;
  const int pre = wave_prefix(m_l, 16, &M);
  uint32_t lists_new = 0;
  for (int s = 0; s < 8; ++s)
    if (__ballot((lbits >> (8 + s)) & 1u)) lists_new |= 1u << s;
  uint64_t dnew = 0;
  if (M > 0) {
    const int64_t words = ((int64_t)M * EW + 3) & ~3ll;
    if (lane == 0) sh_base = ring_alloc(L.head, L.tail[sub], L.ring_cap[sub], sub, words);
    __syncthreads();
    const int64_t base = sh_base;
    if (base < 0) {
      if (lane == 0) atomicOr(&L.err[1], 1);
      return;
    }
    uint32_t* dst = L.ring[sub] + base + (int64_t)pre * EW;
    int t = 0;
    for (int k = b_l; k < e_l; ++k) {
      const uint32_t* e = ent + k * EW;
      if (!((e[0] & EF_INLIST) || (e[0] & EF_MARKER))) continue;
      for (int w = 0; w < EW; ++w) dst[t * EW + w] = e[w];
      ++t;
    }
    for (int k = n_old; k < n_old + n_new; ++k) {
      const uint32_t* e = ent + k * EW;
      if ((int)(e[0] & EF_LANE) != lane) continue;
      for (int w = 0; w < EW; ++w) dst[t * EW + w] = e[w];
      ++t;
    }
    dnew = (uint64_t)(base / 4) | ((uint64_t)M << 40) | ((uint64_t)lists_new << 56);
    if (lane == 0) atomicAdd(&L.traffic[item & 255], (unsigned long long)words * 4);
  }
  // partials (not markers) gained by this block: the live-partial count, spread over 256 counters
  int pn = 0, po = 0;
  (void)wave_prefix(parts_new, 16, &pn);
  (void)wave_prefix(parts_old, 16, &po);
  if (lane == 0) {
    L.journal[item] = d0;
    L.journal_idx[item] = dir_idx;
    L.dir[dir_idx] = dnew;
    if (pn != po) atomicAdd((unsigned long long*)&L.live[item & 255], (unsigned long long)(long long)(pn - po));
  }
}

// A failed push: every directory entry the kernel replaced gets its old value back (the old blocks
// were never written: each changed block went to a new place)
__global__ void slab_rollback_kernel(uint64_t* dir, const uint64_t* journal, const uint64_t* journal_idx, int64_t n,
                                     const long long* live_bak, long long* live) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 256) live[i] = live_bak[i];
  if (i >= n) return;
  if (journal_idx[i] != ~0ull) dir[journal_idx[i]] = journal[i];
}

// Move the blocks of the directory entries [0, n_dir) of the sub-rings marked in `active` whose ring
// position is before limit[sub] (in the source rings) to the head of their ring in the destination:
// reclaiming a ring's oldest blocks (src == dst), growing rings (every block into larger buffers),
// packing for a snapshot (dst_nsub == 1: one ring) or unpacking a snapshot (src_nsub == 1). A block
// keeps its old place until its directory word moves; err[0] = 1 when a destination ring is full.
struct SlabRings {
  uint32_t* const* ring;
  const int64_t* cap;
  unsigned long long* head;
  const unsigned long long* tail;
  int32_t nsub;
};
// One wave per 64 directory entries: each lane decides whether its block moves and takes its
// destination (one ring_alloc), then copies it in 16-B words (a block is a multiple of 4 uint32 words
// at a 16-B aligned offset) if it is small -- C5's blocks mostly are: 64 copies in flight -- while the
// wave copies a large one together, all 64 lanes on it. (A thread copying its own block word by word
// in 4-B loads read 64 scattered lines per instruction.)
__global__ __launch_bounds__(256) void slab_move_kernel(uint64_t* dir, int64_t n_dir, int groups,
                                                        const int32_t* __restrict__ group_ew, SlabRings src,
                                                        const unsigned long long* limit, const uint8_t* active,
                                                        SlabRings dst, int32_t* err, uint8_t* ring_err) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  bool mv = false;
  uint64_t d = 0;
  int64_t words = 0, o = -1;
  const uint32_t* from = nullptr;
  uint32_t* to = nullptr;
  if (x < n_dir) {
    d = dir[x];
    const int n = (int)((d >> 40) & 0xffff);
    const uint32_t ss = src.nsub == 1 ? 0u : sub_of((uint64_t)x, src.nsub);
    if (n != 0 && (!active || active[ss])) {
      const int64_t rel = (int64_t)(d & 0xffffffffull) * 4, cap = src.cap[ss];
      const uint64_t t = src.tail[ss];
      const uint64_t logical = t + (uint64_t)((rel - (int64_t)(t % (uint64_t)cap) + cap) % cap);
      if (logical < limit[ss]) {
        const int64_t g = x < (int64_t)UINT32_MAX ? (int64_t)((uint32_t)x % (uint32_t)groups) : x % groups;
        words = ((int64_t)n * group_ew[g] + 3) & ~3ll;
        const uint32_t ds = dst.nsub == 1 ? 0u : sub_of((uint64_t)x, dst.nsub);
        o = ring_alloc(dst.head, dst.tail[ds], dst.cap[ds], ds, words);
        if (o < 0) {
          atomicOr(err, 1);
          if (ring_err) ring_err[ds] = 1;  // (which destination ring ran out of room)
        } else {
          mv = true;
          from = src.ring[ss] + rel;
          to = dst.ring[ds] + o;
        }
      }
    }
  }
  // a block of up to 32 16-B words: its lane copies it (64 blocks at a time); a larger one: the whole
  // wave, one block after another (a block keeps its old place until its directory word moves)
  const bool own = mv && words <= 4 * 32;
  if (own) {
    const uint4* f = reinterpret_cast<const uint4*>(from);
    uint4* t = reinterpret_cast<uint4*>(to);
    for (int64_t i = 0; i < words / 4; ++i) t[i] = f[i];
  }
  for (unsigned long long m = __ballot(mv && !own); m; m &= m - 1) {
    const int l = __ffsll((long long)m) - 1;
    const uint4* f = reinterpret_cast<const uint4*>(
        (const uint32_t*)__shfl((long long)(uintptr_t)from, l));
    uint4* t = reinterpret_cast<uint4*>((uint32_t*)__shfl((long long)(uintptr_t)to, l));
    const int64_t q = __shfl(words, l) / 4;
    for (int64_t i = lane; i < q; i += 64) t[i] = f[i];
  }
  if (mv) dir[x] = (uint64_t)(o / 4) | (d & ~0xffffffffull);
}

// live words of the blocks (stats: bytes per live partial)
__global__ void slab_live_words_kernel(const uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                       unsigned long long* acc) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long w = 0;
  if (x < n_dir) {
    const uint64_t d = dir[x];
    const int n = (int)((d >> 40) & 0xffff);
    if (n) w = (unsigned long long)(((int64_t)n * group_ew[x % groups] + 3) & ~3ll);
  }
  for (int o = 32; o > 0; o >>= 1) w += __shfl_down(w, o);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(acc, w);
}

// live words per sub-ring (acc[nsub]): a block-local histogram in LDS, one atomic per ring per block
__global__ __launch_bounds__(256) void slab_live_words_ring_kernel(const uint64_t* dir, int64_t n_dir, int groups,
                                                                   const int32_t* group_ew, int nsub,
                                                                   unsigned long long* acc) {
  extern __shared__ unsigned long long hist[];
  for (int i = threadIdx.x; i < nsub; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_dir; x += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t d = dir[x];
    const int n = (int)((d >> 40) & 0xffff);
    if (n)
      atomicAdd(&hist[nsub == 1 ? 0u : sub_of((uint64_t)x, nsub)],
                (unsigned long long)(((int64_t)n * group_ew[x % groups] + 3) & ~3ll));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nsub; i += blockDim.x)
    if (hist[i]) atomicAdd(&acc[i], hist[i]);
}

}  // namespace sdh

extern "C" hipError_t sdh_slab_live_words_ring(const uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                               int nsub, unsigned long long* acc, hipStream_t s) {
  if (n_dir <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>(2048, (n_dir + 255) / 256);
  hipLaunchKernelGGL(sdh::slab_live_words_ring_kernel, dim3((unsigned)blocks), dim3(256), (size_t)nsub * 8, s, dir,
                     n_dir, groups, group_ew, nsub, acc);
  return hipGetLastError();
}

extern "C" hipError_t sdh_launch_slab(const sdh::SlabLaunch* L, hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  const size_t lds = (size_t)L->lds_words * 4;
  const unsigned grid = (unsigned)(L->xcd ? (L->n_items + 7) & ~7 : L->n_items);
  // waves per SIMD the register allocation aims at (SDH_SLAB_WPE; LDS allows ~4 at the small tier)
  const int wpe = sdh::knob("SDH_SLAB_WPE") ? atoi(sdh::knob("SDH_SLAB_WPE")) : 4;
  if (L->max_na <= 4) {
    if (wpe >= 6) hipLaunchKernelGGL((sdh::nfa_slab_kernel<4, 6>), dim3(grid), dim3(64), lds, s, *L);
    else if (wpe == 5) hipLaunchKernelGGL((sdh::nfa_slab_kernel<4, 5>), dim3(grid), dim3(64), lds, s, *L);
    else hipLaunchKernelGGL((sdh::nfa_slab_kernel<4, 1>), dim3(grid), dim3(64), lds, s, *L);
  } else {
    hipLaunchKernelGGL((sdh::nfa_slab_kernel<sdh::kg::GMAXNA, 1>), dim3(grid), dim3(64), lds, s, *L);
  }
  return hipGetLastError();
}

extern "C" hipError_t sdh_slab_rollback(uint64_t* dir, const uint64_t* journal, const uint64_t* journal_idx, int64_t n,
                                        const long long* live_bak, long long* live, hipStream_t s) {
  const int64_t m = n > 256 ? n : 256;
  hipLaunchKernelGGL(sdh::slab_rollback_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, dir, journal,
                     journal_idx, n, live_bak, live);
  return hipGetLastError();
}

extern "C" hipError_t sdh_slab_move(uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                    uint32_t* const* src_ring, const int64_t* src_cap,
                                    const unsigned long long* src_tail, int src_nsub, const unsigned long long* limit,
                                    const uint8_t* active, uint32_t* const* dst_ring, const int64_t* dst_cap,
                                    unsigned long long* dst_head, const unsigned long long* dst_tail, int dst_nsub,
                                    int32_t* err, uint8_t* ring_err, hipStream_t s) {
  if (n_dir <= 0) return hipSuccess;
  const sdh::SlabRings S{src_ring, src_cap, nullptr, src_tail, src_nsub};
  const sdh::SlabRings D{dst_ring, dst_cap, dst_head, dst_tail, dst_nsub};
  hipLaunchKernelGGL(sdh::slab_move_kernel, dim3((unsigned)((n_dir + 255) / 256)), dim3(256), 0, s, dir, n_dir, groups,
                     group_ew, S, limit, active, D, err, ring_err);
  return hipGetLastError();
}

extern "C" hipError_t sdh_slab_live_words(const uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                          unsigned long long* acc, hipStream_t s) {
  if (n_dir <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::slab_live_words_kernel, dim3((unsigned)((n_dir + 255) / 256)), dim3(256), 0, s, dir, n_dir,
                     groups, group_ew, acc);
  return hipGetLastError();
}
