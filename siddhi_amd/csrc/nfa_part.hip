// nfa_part.hip -- K_part (part_body.h: shapes, exactness argument, CDNA4 mapping) with the
// shape's filters interpreted; spec.hip compiles the same body with the filters as straight-line
// code for shapes that fill at least two waves.
#include <hip/hip_runtime.h>

#include "part_body.h"

namespace sdh {

namespace {

__device__ __forceinline__ kg::Val typed(const kg::GInsn& in, int64_t raw, bool isnull) {
  kg::Val v{in.res, 1, 0};
  if (!isnull) {
    v.null = 0;
    v.bits = in.res == kg::T_INT ? (int64_t)(int32_t)raw : in.res == kg::T_FLOAT ? (int64_t)(uint32_t)raw : raw;
  }
  return v;
}

// an event-only filter of state `sid` (FilterProcessor.java:55-66 over the typed bytecode): the
// state's own one-event slot at index 0 / CURRENT is the event, every other reference is null
__device__ __forceinline__ bool ev_filter(const kg::GQuery* q, const kg::GQuery* ql, int sid, const PartEv& ev) {
  const kg::GState& gs = q->st[sid];
  for (int f = 0; f < gs.n_filt; ++f) {
    const kg::Val v = kg::eval_code<kg::RegStack>(
        q, ql, gs.fb[f], gs.fe[f],
        [&](const kg::GInsn& in) {
          const bool here = in.a == sid && (in.b == 0 || in.b == -1);
          return typed(in, here ? ev.word(in.imm) : 0, !here || ev.null(in.imm));
        },
        [&](const kg::GInsn& in) { return !(in.a == sid && (in.b == 0 || in.b == -1)); });
    if (v.null || !v.bits) return false;
  }
  return true;
}

}  // namespace

// K_part with the shape's filters interpreted (the bytecode walked per event)
struct PartInterp {
  static constexpr int kRegEntries = 0, kEW = 1;  // the whole table in the global state block
  static constexpr bool kHotRegs = false;         // (GMAXNA-wide hot rows would not stay in VGPRs)
  static constexpr int kNA = kg::GMAXNA, kOutW = 1536;
  struct K {};
  __device__ static void load(K&, const kg::GQuery*, const PartLaunch&, const int64_t*) {}
  __device__ static PartOffs offs(const PartLaunch& L) { return PartOffs{L.cmax, L.n_e1, L.n_first, L.n_last}; }
  __device__ static bool f1(const K&, const kg::GQuery* q, const kg::GQuery* ql, const PartLaunch&, const PartEv& ev) {
    return ev_filter(q, ql, 0, ev);
  }
  __device__ static bool fa(const K&, const kg::GQuery* q, const kg::GQuery* ql, const PartLaunch& L, const PartEv& ev) {
    return ev_filter(q, ql, L.sA, ev);
  }
  __device__ static bool fb(const K&, const kg::GQuery* q, const kg::GQuery* ql, const PartLaunch& L, const PartEv& ev) {
    return ev_filter(q, ql, L.sB, ev);
  }
  __device__ static bool f2(const K&, const kg::GQuery* q, const kg::GQuery* ql, const PartLaunch&, const PartEv& ev) {
    return ev_filter(q, ql, 1, ev);
  }
  // e3 of the count chain over the partial as it is now: slot 2 the current event, slot 0 e1,
  // slot 1 the chain's first (index 0) or last (CURRENT) event -- all exist (len >= min >= 1)
  template <class En>
  __device__ static bool f3(const K&, const kg::GQuery* q, const kg::GQuery* ql, const PartLaunch&, const PartEv& ev,
                            const En& en) {
    const kg::GState& s3 = q->st[2];
    for (int f = 0; f < s3.n_filt; ++f) {
      const kg::Val v = kg::eval_code<kg::RegStack>(
          q, ql, s3.fb[f], s3.fe[f],
          [&](const kg::GInsn& in) {
            const bool here = in.b == 0 || in.b == -1;
            if (in.a == 2) return typed(in, here ? ev.word(in.imm) : 0, !here || ev.null(in.imm));
            if (in.a == 0) return typed(in, here ? en.e1(in.imm) : 0, !here || en.e1_null(in.imm));
            const bool first = in.b == 0;
            return typed(in, first ? en.first(in.imm) : en.last(in.imm),
                         first ? en.first_null(in.imm) : en.last_null(in.imm));
          },
          [&](const kg::GInsn&) { return false; });
      if (v.null || !v.bits) return false;
    }
    return true;
  }
};

template <int KIND>
__global__ __launch_bounds__(64) void nfa_part_kernel(PartLaunch L) {
  part_body<KIND, PartInterp>(L);
}

// live partials (sdh_engine_stats): table entries in each key's current buffer; one thread per
// (key, group, lane)
// the batch in key order (position t <- batch event idx[t]): ts, every column, every null mask
__global__ __launch_bounds__(256) void sort_batch_kernel(StreamBatch b, const int32_t* __restrict__ idx, StreamBatch o) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= b.n) return;
  const int64_t e = idx[t];
  const_cast<int64_t*>(o.ts)[t] = b.ts[e];
  for (int a = 0; a < b.n_attr; ++a) {
    const int w = b.width[a];
    if (w == 8) ((int64_t*)o.col[a])[t] = ((const int64_t*)b.col[a])[e];
    else if (w == 4) ((int32_t*)o.col[a])[t] = ((const int32_t*)b.col[a])[e];
    else ((uint8_t*)o.col[a])[t] = ((const uint8_t*)b.col[a])[e];
    if (b.nul[a]) const_cast<uint8_t*>(o.nul[a])[t] = b.nul[a][e];
  }
}

__global__ void part_live_kernel(const int64_t* __restrict__ st, const int32_t* __restrict__ cur, int64_t n_keys,
                                 int groups, int64_t blocks, int64_t bw, unsigned long long* acc) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t blk = x >> 6;
  unsigned long long v = 0;
  if (blk / groups < n_keys) {
    const int64_t kid = blk / groups;
    v = (unsigned long long)st[(((int64_t)cur[kid] * blocks + blk) * bw) * 64 + (x & 63)];
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(acc, v);
}

}  // namespace sdh

// bytes the key-ordered copy of a batch takes (256-B aligned parts), and the copy itself: `o` gets
// the same schema with its pointers into buf
extern "C" size_t sdh_sorted_batch_bytes(const sdh::StreamBatch* b) {
  size_t t = ((size_t)b->n * 8 + 255) & ~(size_t)255;
  for (int a = 0; a < b->n_attr; ++a) {
    t += ((size_t)b->n * b->width[a] + 255) & ~(size_t)255;
    if (b->nul[a]) t += ((size_t)b->n + 255) & ~(size_t)255;
  }
  return t;
}
extern "C" hipError_t sdh_sort_batch(const sdh::StreamBatch* b, const int32_t* idx, uint8_t* buf, sdh::StreamBatch* o,
                                     hipStream_t s) {
  *o = *b;
  size_t t = 0;
  auto take = [&](size_t bytes) {
    uint8_t* p = buf + t;
    t += (bytes + 255) & ~(size_t)255;
    return p;
  };
  o->ts = (const int64_t*)take((size_t)b->n * 8);
  for (int a = 0; a < b->n_attr; ++a) {
    o->col[a] = take((size_t)b->n * b->width[a]);
    o->nul[a] = b->nul[a] ? take((size_t)b->n) : nullptr;
  }
  if (b->n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::sort_batch_kernel, dim3((unsigned)((b->n + 255) / 256)), dim3(256), 0, s, *b, idx, *o);
  return hipGetLastError();
}

extern "C" hipError_t sdh_live_part(const int64_t* st, const int32_t* cur, int64_t n_keys, int groups, int64_t blocks,
                                    int64_t bw, unsigned long long* acc, hipStream_t s) {
  const int64_t threads = n_keys * groups * 64;
  if (threads <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::part_live_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, st, cur, n_keys,
                     groups, blocks, bw, acc);
  return hipGetLastError();
}

extern "C" hipError_t sdh_launch_part(const sdh::PartLaunch* L, hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  const dim3 grid(L->xcd ? (L->n_items + 7) & ~7 : L->n_items);
  switch (L->kind) {
    case sdh::PK_OR: hipLaunchKernelGGL(sdh::nfa_part_kernel<sdh::PK_OR>, grid, dim3(64), 0, s, *L); break;
    case sdh::PK_AND: hipLaunchKernelGGL(sdh::nfa_part_kernel<sdh::PK_AND>, grid, dim3(64), 0, s, *L); break;
    default: hipLaunchKernelGGL(sdh::nfa_part_kernel<sdh::PK_COUNT>, grid, dim3(64), 0, s, *L);
  }
  return hipGetLastError();
}
