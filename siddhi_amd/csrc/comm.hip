// comm.hip -- the multi-GPU exchange (comm.h): RCCL and in-process transports, and the device k-way
// merge of the per-rank match runs.
//
// Reference order the merge keeps: a StreamJunction hands each event to its receivers in
// subscription order (stream/StreamJunction.java:179-181), and a partitioned event goes to the one
// partition key that owns it (stream/output/sink/distributed/PartitionedDistributionStrategy.java:
// 98-109 is the destination rule the key shards follow). Each rank's matches come out of its own
// poll already in R18 order, sorted by the poll's key (chunk keys, trigger seq << 20 | receiver rank,
// timer tiebreaks); rows of different ranks never tie on that key (a receiver's matches of one event
// come from one rank: its pattern shard, or the owner of the event's key), so the single-engine
// order is a k-way merge of the runs.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/siddhi_hip.h"
#include "comm.h"

namespace {

struct LocalGroup {
  std::mutex mu;
  struct Slot {
    // broadcasts this rank published as root (gen counts them), and the last one it consumed
    uint64_t bgen = 0;
    std::vector<uint64_t> seen_hdr, seen_bufs;  // [root]
    int64_t bhdr[sdh::xch::HDR] = {};
    std::vector<sdh::xch::Buf> bbufs;
    uint64_t bbufs_gen = 0;
    // this rank's gather deposit (non-root ranks), taken by rank 0
    bool g_hdr = false, g_bufs = false;
    int64_t ghdr[sdh::xch::HDR] = {};
    std::vector<sdh::xch::Buf> gbufs;
    // stream order between ranks: the depositing rank records an event on its stream once its buffers
    // are complete (a broadcast root's batch, a gather deposit), and the copying rank's stream waits on
    // it before its copies (raw pointers alone carry no ordering)
    hipEvent_t bev = nullptr, gev = nullptr;
  };
  std::vector<Slot> slots;
  ~LocalGroup() {
    for (auto& sl : slots) {
      if (sl.bev) (void)hipEventDestroy(sl.bev);
      if (sl.gev) (void)hipEventDestroy(sl.gev);
    }
  }
};

[[noreturn]] void fail(const std::string& m) { throw std::runtime_error(m); }
// a local-communicator call out of order (a caller error, not a transport failure)
[[noreturn]] void misuse(const std::string& m) { throw std::invalid_argument(m); }

void hipchk(hipError_t e, const char* what) {
  if (e != hipSuccess) fail(std::string(what) + ": " + hipGetErrorString(e));
}
// record `ev` (created on first use, on the calling rank's device) on stream s
void mark(hipEvent_t& ev, hipStream_t s) {
  if (!ev) hipchk(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  hipchk(hipEventRecord(ev, s), "hipEventRecord");
}
void ncclchk(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) fail(std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

struct sdh_comm {
  bool local = false;
  int rank = 0, world = 1, device = 0;
  ncclComm_t nc = nullptr;
  std::shared_ptr<LocalGroup> grp;
  int64_t* scratch = nullptr;  // RCCL: world x HDR header words in HBM
  ~sdh_comm() {
    if (nc) (void)ncclCommDestroy(nc);
    if (scratch) (void)hipFree(scratch);
  }
};

namespace sdh {
namespace xch {

int rank(const sdh_comm* c) { return c->rank; }
bool is_local(const sdh_comm* c) { return c->local; }
int world(const sdh_comm* c) { return c->world; }
int device(const sdh_comm* c) { return c->device; }

void bcast_hdr(sdh_comm* c, int64_t hdr[HDR], int root, hipStream_t s) {
  if (root < 0 || root >= c->world) misuse("broadcast root out of range");
  if (c->local) {
    std::lock_guard<std::mutex> g(c->grp->mu);
    auto& R = c->grp->slots[(size_t)root];
    auto& me = c->grp->slots[(size_t)c->rank];
    if (c->rank == root) {
      for (int r = 0; r < c->world; ++r)  // (the previous batch reached every rank before this one)
        if (r != root && R.bgen && c->grp->slots[(size_t)r].seen_hdr[(size_t)root] != R.bgen)
          misuse("local communicator: rank " + std::to_string(r) + " has not received the root's previous batch");
      ++R.bgen;
      std::memcpy(R.bhdr, hdr, sizeof R.bhdr);
      R.bbufs.clear();
      R.bbufs_gen = 0;
      return;
    }
    if (R.bgen == 0 || me.seen_hdr[(size_t)root] == R.bgen)
      misuse("local communicator: the broadcast root has not pushed this batch yet (root first)");
    std::memcpy(hdr, R.bhdr, sizeof R.bhdr);
    me.seen_hdr[(size_t)root] = R.bgen;
    return;
  }
  // (RCCL at world 1 too: the collective runs, copying in place)
  hipchk(hipMemcpyAsync(c->scratch, hdr, HDR * 8, hipMemcpyHostToDevice, s), "broadcast header");
  ncclchk(ncclBroadcast(c->scratch, c->scratch, HDR, ncclInt64, root, c->nc, s), "ncclBroadcast (header)");
  hipchk(hipMemcpyAsync(hdr, c->scratch, HDR * 8, hipMemcpyDeviceToHost, s), "broadcast header");
  hipchk(hipStreamSynchronize(s), "broadcast header");
}

void bcast_bufs(sdh_comm* c, const std::vector<Buf>& bufs, int root, hipStream_t s) {
  if (c->local) {
    std::lock_guard<std::mutex> g(c->grp->mu);
    auto& R = c->grp->slots[(size_t)root];
    auto& me = c->grp->slots[(size_t)c->rank];
    if (c->rank == root) {
      R.bbufs = bufs;
      R.bbufs_gen = R.bgen;
      mark(R.bev, s);
      return;
    }
    if (R.bbufs_gen != me.seen_hdr[(size_t)root] || R.bbufs.size() != bufs.size() ||
        me.seen_bufs[(size_t)root] == R.bbufs_gen)
      misuse("local communicator: broadcast buffers out of step with the root");
    hipchk(hipStreamWaitEvent(s, R.bev, 0), "hipStreamWaitEvent");
    for (size_t i = 0; i < bufs.size(); ++i) {
      if (R.bbufs[i].bytes != bufs[i].bytes) misuse("local communicator: broadcast buffer sizes differ");
      if (bufs[i].bytes)
        hipchk(hipMemcpyAsync(bufs[i].dst, R.bbufs[i].src, bufs[i].bytes, hipMemcpyDefault, s), "broadcast copy");
    }
    me.seen_bufs[(size_t)root] = R.bbufs_gen;
    return;
  }
  ncclchk(ncclGroupStart(), "ncclGroupStart");
  for (const Buf& b : bufs) {
    if (!b.bytes) continue;
    void* p = c->rank == root ? const_cast<void*>(b.src) : b.dst;
    ncclchk(ncclBroadcast(p, p, b.bytes, ncclUint8, root, c->nc, s), "ncclBroadcast");
  }
  ncclchk(ncclGroupEnd(), "ncclGroupEnd");
}

void gather_hdr(sdh_comm* c, const int64_t hdr[HDR], int64_t* all, hipStream_t s) {
  if (c->local) {
    std::lock_guard<std::mutex> g(c->grp->mu);
    auto& me = c->grp->slots[(size_t)c->rank];
    if (c->rank != 0) {
      if (me.g_hdr) misuse("local communicator: rank 0 has not taken this rank's previous gather");
      std::memcpy(me.ghdr, hdr, sizeof me.ghdr);
      me.g_hdr = true;
      me.g_bufs = false;
      return;
    }
    std::memcpy(all, hdr, HDR * 8);
    for (int r = 1; r < c->world; ++r) {
      auto& S = c->grp->slots[(size_t)r];
      if (!S.g_hdr) misuse("local communicator: rank " + std::to_string(r) + " has not gathered yet (rank 0 last)");
      std::memcpy(all + (size_t)r * HDR, S.ghdr, HDR * 8);
    }
    return;
  }
  // RCCL: an all-gather, so that every rank sees every header and can refuse an out-of-step window
  // before any rank clears its table or sends its buffers (world 1 included)
  int64_t* mine = c->scratch + (size_t)c->world * HDR;
  hipchk(hipMemcpyAsync(mine, hdr, HDR * 8, hipMemcpyHostToDevice, s), "gather header");
  ncclchk(ncclAllGather(mine, c->scratch, HDR, ncclInt64, c->nc, s), "ncclAllGather (header)");
  hipchk(hipMemcpyAsync(all, c->scratch, (size_t)c->world * HDR * 8, hipMemcpyDeviceToHost, s), "gather header");
  hipchk(hipStreamSynchronize(s), "gather header");
}

void gather_bufs(sdh_comm* c, const std::vector<Buf>& mine, const std::vector<std::vector<Buf>>& recv, hipStream_t s) {
  if (c->local) {
    std::lock_guard<std::mutex> g(c->grp->mu);
    if (c->rank != 0) {
      auto& me = c->grp->slots[(size_t)c->rank];
      me.gbufs = mine;
      me.g_bufs = true;
      mark(me.gev, s);
      return;
    }
    for (int r = 1; r < c->world; ++r) {
      auto& S = c->grp->slots[(size_t)r];
      const auto& want = recv[(size_t)r];
      if (!S.g_bufs || S.gbufs.size() != want.size()) misuse("local communicator: gather buffers out of step");
      hipchk(hipStreamWaitEvent(s, S.gev, 0), "hipStreamWaitEvent");
      for (size_t i = 0; i < want.size(); ++i) {
        if (S.gbufs[i].bytes != want[i].bytes) misuse("local communicator: gather buffer sizes differ");
        if (want[i].bytes)
          hipchk(hipMemcpyAsync(want[i].dst, S.gbufs[i].src, want[i].bytes, hipMemcpyDefault, s), "gather copy");
      }
      S.g_hdr = S.g_bufs = false;
    }
    return;
  }
  // RCCL: every rank sends its run to rank 0 -- rank 0 to itself as well (a self send / receive, so
  // world 1 runs the same transfers), and rank 0 receives every rank's
  ncclchk(ncclGroupStart(), "ncclGroupStart");
  for (const Buf& b : mine)
    if (b.bytes) ncclchk(ncclSend(b.src, b.bytes, ncclUint8, 0, c->nc, s), "ncclSend");
  if (c->rank == 0)
    for (int r = 0; r < c->world; ++r)
      for (const Buf& b : recv[(size_t)r])
        if (b.bytes) ncclchk(ncclRecv(b.dst, b.bytes, ncclUint8, r, c->nc, s), "ncclRecv");
  ncclchk(ncclGroupEnd(), "ncclGroupEnd");
}

}  // namespace xch
}  // namespace sdh

// ---- the device k-way merge ----
namespace {

constexpr int MAX_KW = 6;

struct Runs {  // (by value: the kernels read it from the argument segment)
  int64_t off[SDH_MAX_RANKS + 1];
  int64_t wbase[SDH_MAX_RANKS];
  int k;
};

__device__ __forceinline__ int run_of(const Runs& R, int64_t i) {
  int r = 0;
  while (r + 1 < R.k && R.off[r + 1] <= i) ++r;
  return r;
}

// rows of [b, e) whose key is below x (upper: or equal)
__device__ int64_t rows_before(const uint64_t* __restrict__ keys, int kw, int64_t b, int64_t e, const uint64_t* x,
                               bool upper) {
  int64_t lo = b, hi = e;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    const uint64_t* y = keys + mid * kw;
    int c = 0;
    for (int w = 0; w < kw && c == 0; ++w) c = y[w] < x[w] ? -1 : y[w] > x[w] ? 1 : 0;
    if (c < 0 || (upper && c == 0)) lo = mid + 1;
    else hi = mid;
  }
  return lo - b;
}

// a row's output position: its index in its run plus, per other run, the rows ordered before it
// (an earlier run's equal keys too: ties keep run order, as a stable sort of the concatenation)
__global__ __launch_bounds__(256) void merge_pos_kernel(const uint64_t* __restrict__ keys, int kw, Runs R, int64_t N,
                                                        int64_t* __restrict__ pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int r = run_of(R, i);
  uint64_t x[MAX_KW];
  for (int w = 0; w < kw; ++w) x[w] = keys[i * kw + w];
  int64_t p = i - R.off[r];
  for (int r2 = 0; r2 < R.k; ++r2)
    if (r2 != r && R.off[r2 + 1] > R.off[r2]) p += rows_before(keys, kw, R.off[r2], R.off[r2 + 1], x, r2 < r);
  pos[i] = p;
}

__global__ __launch_bounds__(256) void merge_scatter_kernel(Runs R, int64_t N, const int64_t* __restrict__ pos,
                                                            const int64_t* __restrict__ q, const int64_t* __restrict__ key,
                                                            const int64_t* __restrict__ ts, const int64_t* __restrict__ seq,
                                                            const int64_t* __restrict__ tb,
                                                            const int64_t* __restrict__ off_cat, int64_t* __restrict__ oq,
                                                            int64_t* __restrict__ okey, int64_t* __restrict__ ots,
                                                            int64_t* __restrict__ oseq, int64_t* __restrict__ otb,
                                                            int64_t* __restrict__ olen, int64_t* __restrict__ osrc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > N) return;
  if (i == N) {
    olen[N] = 0;
    return;
  }
  const int r = run_of(R, i);
  const int64_t j = i - R.off[r];
  const int64_t* o = off_cat + R.off[r] + r;
  const int64_t p = pos[i];
  oq[p] = q[i];
  okey[p] = key[i];
  ots[p] = ts[i];
  oseq[p] = seq[i];
  otb[p] = tb[i];
  olen[p] = o[j + 1] - o[j];
  osrc[p] = R.wbase[r] + o[j];
}

__global__ __launch_bounds__(256) void merge_words_kernel(const int64_t* __restrict__ osrc,
                                                          const int64_t* __restrict__ ooff, int64_t N,
                                                          const int64_t* __restrict__ words,
                                                          int64_t* __restrict__ owords) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int64_t* s = words + osrc[i];
  int64_t* d = owords + ooff[i];
  const int64_t len = ooff[i + 1] - ooff[i];
  for (int64_t k = 0; k < len; ++k) d[k] = s[k];
}

inline unsigned grid(int64_t n) { return (unsigned)((n + 255) / 256); }

thread_local std::string g_comm_error;

int comm_fail(const std::exception& ex) {
  g_comm_error = ex.what();
  return SDH_E_DEVICE;
}

}  // namespace

extern "C" size_t sdh_merge_temp_bytes(int64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n + 1));
  return b + 256;
}

extern "C" hipError_t sdh_merge_runs(const uint64_t* keys, int kw, const int64_t* run_off, int k, int64_t N,
                                     const int64_t* q, const int64_t* key, const int64_t* ts, const int64_t* seq,
                                     const int64_t* tb, const int64_t* off_cat, const int64_t* word_base,
                                     int64_t* pos, int64_t* oq, int64_t* okey, int64_t* ots, int64_t* oseq,
                                     int64_t* otb, int64_t* olen, int64_t* ooff, int64_t* osrc, void* temp,
                                     size_t temp_bytes, int64_t* total_words, hipStream_t s) {
  *total_words = 0;
  if (k < 1 || k > SDH_MAX_RANKS || kw < 1 || kw > MAX_KW || N >= INT32_MAX) return hipErrorInvalidValue;
  Runs R{};
  R.k = k;
  for (int r = 0; r <= k; ++r) R.off[r] = run_off[r];
  for (int r = 0; r < k; ++r) R.wbase[r] = word_base[r];
  if (N > 0) hipLaunchKernelGGL(merge_pos_kernel, dim3(grid(N)), dim3(256), 0, s, keys, kw, R, N, pos);
  hipLaunchKernelGGL(merge_scatter_kernel, dim3(grid(N + 1)), dim3(256), 0, s, R, N, pos, q, key, ts, seq, tb, off_cat,
                     oq, okey, ots, oseq, otb, olen, osrc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb2 = temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(temp, tb2, olen, ooff, (int)(N + 1), s);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(total_words, ooff + N, 8, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(s);
}

extern "C" hipError_t sdh_merge_words(const int64_t* osrc, const int64_t* ooff, int64_t N, const int64_t* words,
                                      int64_t* owords, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_words_kernel, dim3(grid(N)), dim3(256), 0, s, osrc, ooff, N, words, owords);
  return hipGetLastError();
}

// ---- ABI (include/siddhi_hip.h) ----
extern "C" {

int sdh_comm_get_id(void* id, size_t cap) {
  if (!id || cap < SDH_COMM_ID_BYTES) return SDH_E_INVALID;
  static_assert(SDH_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    g_comm_error = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return SDH_E_DEVICE;
  }
  std::memcpy(id, &u, SDH_COMM_ID_BYTES);
  return SDH_OK;
}

int sdh_comm_create(const void* id, size_t len, int32_t rank, int32_t world, int32_t device, sdh_comm** out) {
  if (!out) return SDH_E_INVALID;
  *out = nullptr;
  if (!id || len < SDH_COMM_ID_BYTES || world < 1 || world > SDH_MAX_RANKS || rank < 0 || rank >= world) {
    g_comm_error = "sdh_comm_create: bad id, rank or world";
    return SDH_E_INVALID;
  }
  try {
    std::unique_ptr<sdh_comm> c(new sdh_comm);
    c->rank = rank;
    c->world = world;
    c->device = device;
    hipchk(hipSetDevice(device), "hipSetDevice");
    hipchk(hipMalloc(&c->scratch, (size_t)(world + 1) * sdh::xch::HDR * 8), "hipMalloc");
    ncclUniqueId u;
    std::memcpy(&u, id, SDH_COMM_ID_BYTES);
    ncclchk(ncclCommInitRank(&c->nc, world, u, rank), "ncclCommInitRank");
    *out = c.release();
    return SDH_OK;
  } catch (const std::exception& ex) {
    return comm_fail(ex);
  }
}

int sdh_comm_create_local(int32_t world, const int32_t* devices, sdh_comm** out) {
  if (!out || world < 1 || world > SDH_MAX_RANKS) {
    g_comm_error = "sdh_comm_create_local: bad world";
    return SDH_E_INVALID;
  }
  auto grp = std::make_shared<LocalGroup>();
  grp->slots.resize((size_t)world);
  for (auto& sl : grp->slots) {
    sl.seen_hdr.assign((size_t)world, 0);
    sl.seen_bufs.assign((size_t)world, 0);
  }
  for (int r = 0; r < world; ++r) {
    out[r] = new sdh_comm;
    out[r]->local = true;
    out[r]->rank = r;
    out[r]->world = world;
    out[r]->device = devices ? devices[r] : 0;
    out[r]->grp = grp;
  }
  return SDH_OK;
}

void sdh_comm_destroy(sdh_comm* c) { delete c; }

const char* sdh_comm_last_error(void) { return g_comm_error.c_str(); }

}  // extern "C"
