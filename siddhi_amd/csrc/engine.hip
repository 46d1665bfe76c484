// engine.hip -- host side of libsiddhi_hip.so: IR lowering, HBM state management, batching,
// chunk planning, NFA-step launches and match hand-off. Implements include/siddhi_hip.h.
//
// The reference has no device boundary; this file is the GpuStateStreamRuntime half that replaces
// StateInputStreamParser's object graph (core/util/parser/StateInputStreamParser.java:77-398) with
// device tables, and the receiver loop (core/query/input/*ProcessStreamReceiver.java) with one
// batched launch per pushed event batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <tuple>
#include <array>
#include <cmath>
#include <map>
#include <unordered_map>
#include <memory>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/siddhi_hip.h"
#include "chm_order.h"
#include "comm.h"
#include "knobs.h"
#include "java_fmt.h"
#include "gen_lower.h"
#include "nfa_types.h"
#include "slab_lower.h"
#include "spec.h"

extern "C" hipError_t sdh_launch_gen(const sdh::GenLaunch* L, hipStream_t s);
extern "C" hipError_t sdh_launch_part(const sdh::PartLaunch* L, hipStream_t s);
extern "C" hipError_t sdh_launch_seq(const sdh::SeqLaunch* L, hipStream_t s);
extern "C" hipError_t sdh_launch_slab(const sdh::SlabLaunch* L, hipStream_t s);
extern "C" hipError_t sdh_slab_rollback(uint64_t* dir, const uint64_t* journal, const uint64_t* journal_idx, int64_t n,
                                        const long long* live_bak, long long* live, hipStream_t s);
extern "C" hipError_t sdh_slab_move(uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                    uint32_t* const* src_ring, const int64_t* src_cap,
                                    const unsigned long long* src_tail, int src_nsub, const unsigned long long* limit,
                                    const uint8_t* active, uint32_t* const* dst_ring, const int64_t* dst_cap,
                                    unsigned long long* dst_head, const unsigned long long* dst_tail, int dst_nsub,
                                    int32_t* err, uint8_t* ring_err, hipStream_t s);
extern "C" hipError_t sdh_slab_live_words_ring(const uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                               int nsub, unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_slab_live_words(const uint64_t* dir, int64_t n_dir, int groups, const int32_t* group_ew,
                                          unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_seq_tail(const sdh::StreamBatch* b, int64_t* tail, int32_t tail_len, int32_t new_tail_len,
                                   hipStream_t s);
extern "C" hipError_t sdh_route_partition(const sdh::StreamBatch* B, int attr, int type, unsigned long long* tkey,
                                          int32_t* tid, int64_t table_mask, int32_t* n_keys, int64_t* key_of_id,
                                          int64_t key_cap, int64_t* key, uint32_t* kid, uint32_t* kid_sorted,
                                          int32_t* idx, int32_t* idx_sorted, uint32_t* uniq, int32_t* cnt,
                                          int32_t* off, int32_t* n_runs_dev, void* temp, size_t temp_bytes,
                                          int32_t* err, int shard_rank, int shard_world, hipStream_t s);
extern "C" size_t sdh_route_temp_bytes(int64_t n);
extern "C" hipError_t sdh_gen_remap(const int32_t* lane_q, int group_base, int n_groups, int64_t blocks,
                                    const sdh::kg::GLayout* oldL, const sdh::kg::GLayout* newL, const int32_t* o32,
                                    const int64_t* o64, int64_t oB32, int64_t oB64, int32_t* n32, int64_t* n64,
                                    int64_t nB32, int64_t nB64, hipStream_t s);

extern "C" hipError_t sdh_launch_chain(int n_states, int k, const sdh::ChainLaunch* L, int n_blocks,
                                       size_t lds, hipStream_t s);
extern "C" hipError_t sdh_launch_ratchet(int key_kind, int xmask, int full, int nf, int sim, int ML, int SC,
                                         const sdh::RatchetLaunch* L, hipStream_t s);
extern "C" int sdh_ratchet_occupancy(int key_kind, int full, int nf, int ML, int sim);
extern "C" hipError_t sdh_launch_ratchet_summary(int key_kind, const sdh::StreamBatch* B, int attr, int conv,
                                                 int64_t n_tiles, uint64_t* tmax, uint64_t* tmin, uint8_t* thas,
                                                 hipStream_t s);
extern "C" hipError_t sdh_append_ratchet(const int64_t* match, int blk_recs, int wide, const int32_t* blk_count,
                                         const int32_t* blk_group, const int64_t* dst_off,
                                         const sdh::RatchetGroup* groups, const int64_t* ts, int64_t seq_base,
                                         int64_t seq_ref, const int32_t* out_rank, int n_streams, int n_blocks,
                                         sdh::MatchTable T, int64_t row0, int64_t word0, hipStream_t s);
extern "C" hipError_t sdh_append_chain(const int64_t* src, const int64_t* seg_off, const int64_t* seg_count,
                                       const int64_t* dst_off, int rec_words, int n_items, const int32_t* qinfo,
                                       int64_t seq_ref, const int32_t* out_rank, int n_streams, sdh::MatchTable T,
                                       int64_t row0, int64_t word0, hipStream_t s);
extern "C" size_t sdh_gen_words_temp_bytes(int64_t n_rec);
extern "C" size_t sdh_sorted_batch_bytes(const sdh::StreamBatch* b);
extern "C" hipError_t sdh_sort_batch(const sdh::StreamBatch* b, const int32_t* idx, uint8_t* buf, sdh::StreamBatch* o,
                                     hipStream_t s);
extern "C" hipError_t sdh_gen_words(const int64_t* out, const int64_t* rec_off, int64_t n_rec, int64_t* tw, void* temp,
                                    size_t temp_bytes, unsigned long long* n_wide, hipStream_t s);
extern "C" size_t sdh_ex_temp_bytes(int64_t n);
extern "C" hipError_t sdh_ex_chain_words(sdh::MatchTable T, const int32_t* perm, int64_t n, int64_t* cw, void* temp,
                                         size_t temp_bytes, hipStream_t s);
extern "C" hipError_t sdh_ex_rows(sdh::MatchTable T, const int32_t* perm, int64_t n, int width, int64_t seq_ref,
                                  const int64_t* coff, int32_t* rows, int32_t* chain, int64_t* okey, int64_t* otb,
                                  int32_t* err, hipStream_t s);
extern "C" hipError_t sdh_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
extern "C" hipError_t sdh_append_gen(const int64_t* out, const int64_t* rec_off, int64_t n_rec, int64_t seq_ref,
                                     const int32_t* out_rank, const int32_t* fan_rank, int n_streams, sdh::MatchTable T,
                                     int64_t row0, int64_t word0, const int64_t* woff, const int64_t* bts,
                                     int64_t seq_base, int bstream, const int64_t* const* qkeys, hipStream_t s);
extern "C" hipError_t sdh_new_keys(const uint32_t* uniq, const int32_t* nruns, int64_t max_runs, const int32_t* off,
                                   const int32_t* idx_s, const int64_t* key_of_id, int64_t old_n, int64_t new_n,
                                   int64_t* out, hipStream_t s);
extern "C" size_t sdh_poll_temp_bytes(int64_t n);
extern "C" hipError_t sdh_gen_journal(int32_t* a32, int64_t* a64, int64_t B32, int64_t B64, int mode,
                                       const int32_t* glist, const uint32_t* seg_kid, int groups, int64_t slots,
                                       int32_t* j32, int64_t* j64, int64_t* jidx, int restore, hipStream_t s);
extern "C" size_t sdh_place_temp_bytes(int64_t cells);
extern "C" size_t sdh_prefix_max_temp_bytes(int64_t n);
extern "C" hipError_t sdh_prefix_max(const int64_t* ts, int64_t n, int64_t* pm, int32_t* unordered, void* temp,
                                     size_t temp_bytes, hipStream_t s);
extern "C" hipError_t sdh_key_segments(const uint32_t* uniq, const int32_t* nruns, int64_t max_runs, int64_t n_keys,
                                       int32_t* kseg, hipStream_t s);
extern "C" hipError_t sdh_digest_compact(const int32_t* crow, int width, int64_t row0, int64_t n, int64_t seq_ref,
                                         unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_place_scan(int32_t* cnt, int64_t cells, void* temp, size_t temp_bytes, hipStream_t s);
extern "C" hipError_t sdh_merge_keys_table(sdh::MatchTable T, const int32_t* perm, int64_t n, int chunk_words,
                                           int lo_words, int chunked, uint64_t* keys, hipStream_t s);
extern "C" hipError_t sdh_merge_keys_placed(const int32_t* crow, int width, int64_t n, int64_t seq_ref,
                                            const int32_t* out_rank, const int32_t* qinfo, int n_streams,
                                            int chunk_words, int lo_words, uint64_t* keys, hipStream_t s);
extern "C" hipError_t sdh_place_total(const int32_t* cnt, int64_t cells, unsigned long long* tot, hipStream_t s);
extern "C" hipError_t sdh_compact_fill(const int32_t* crow, int width, int64_t rows, const int64_t* ts_log,
                                       int64_t seq_ref, int64_t* oq, int64_t* okey, int64_t* ots, int64_t* oseq,
                                       int64_t* otb, int64_t* ooff, int64_t* owords, hipStream_t s);
extern "C" hipError_t sdh_placed_to_table(const int32_t* crow, int width, int64_t n, const int64_t* ts_log,
                                          int64_t seq_ref, const int32_t* out_rank, const int32_t* qinfo,
                                          int n_streams, sdh::MatchTable T, hipStream_t s);
extern "C" hipError_t sdh_table_compact(sdh::MatchTable T, const int32_t* perm, int64_t n, int width, int64_t seq_ref,
                                        int32_t* crow, int32_t* err, hipStream_t s);
extern "C" hipError_t sdh_live_gen(const int32_t* a32, int64_t B32, int64_t blocks, int n_groups, int group_base,
                                    const int32_t* lane_q, const int32_t* group_seq, const sdh::kg::GQuery* queries,
                                    unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_live_seq(const int64_t* tail, int tail_len, int stream, const int32_t* groups, int n_groups,
                                   const int32_t* lane_q, const int32_t* group_tmpl, const sdh::kg::GQuery* queries,
                                   unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_live_part(const int64_t* st, const int32_t* cur, int64_t n_keys, int groups, int64_t blocks,
                                    int64_t bw, unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_digest_ratchet(const int64_t* match, int blk_recs, int wide, const int32_t* blk_count,
                                         const int32_t* blk_group, const int32_t* blk_side,
                                         const sdh::RatchetGroup* groups, int64_t seq_base,
                                         int n_blocks, unsigned long long* acc, hipStream_t s);
extern "C" hipError_t sdh_launch_gate(int key_kind, int xmask, int full, int nf, int ng, int SC,
                                      const sdh::RatchetLaunch* L, hipStream_t s);
extern "C" int sdh_gate_occupancy(int nf, int ng);
extern "C" size_t sdh_ratchet_compact_temp(int64_t n_blocks);
extern "C" hipError_t sdh_ratchet_compact(const int64_t* match, int blk_recs, int wide, const int32_t* blk_count,
                                          const int32_t* blk_group, const int32_t* blk_side,
                                          const sdh::RatchetGroup* groups, int64_t seq_base, int n_blocks,
                                          int64_t* row_off, void* temp, size_t temp_bytes, int width, int32_t* rows,
                                          hipStream_t s);
extern "C" hipError_t sdh_poll_sort(sdh::MatchTable T, int64_t n, int n_lo, int lo_bits, int hi_bits, int clo_bits,
                                    uint64_t* kbuf, int32_t* pbuf, void* temp, size_t temp_bytes, int64_t* oq,
                                    int64_t* okey, int64_t* ots, int64_t* oseq, int64_t* otb, int64_t* olen,
                                    int64_t* ooff, int32_t** perm_out, int64_t* total_words, hipStream_t s);
extern "C" hipError_t sdh_chunk_keys(sdh::MatchTable T, int64_t r0, int64_t r1, int chunk, int64_t cseq,
                                     int64_t first_seq, int stream, int n_streams, const int32_t* major,
                                     const int32_t* minor, const int32_t* qslot, const int32_t* runs,
                                     int64_t n_events, hipStream_t s);
extern "C" hipError_t sdh_poll_words(sdh::MatchTable T, const int32_t* perm, int64_t n, const int64_t* ooff,
                                     int64_t* owords, hipStream_t s);

using namespace sdh;

namespace {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

std::string fmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) throw Error(SDH_E_DEVICE, fmt("%s: %s", #x, hipGetErrorString(e_))); \
  } while (0)

// ------------------------------------------------------------------------------------------
// IR reader (format: siddhi_amd/ir.py)
// ------------------------------------------------------------------------------------------
enum { OP_CONST = 1, OP_ATTR, OP_IS_NULL, OP_STREAM_IS_NULL, OP_CMP, OP_AND, OP_OR, OP_NOT, OP_ARITH };
enum { K_STREAM = 0, K_COUNT, K_LOGICAL };
enum { Q_PATTERN = 0, Q_SEQUENCE };

struct Insn {
  int op, lt, rt, res;
  int64_t a, b, imm;
};
struct IState {
  int kind, stream, is_start, min, max, ltype, partner, next_pre, next_every, within_every, callback,
      this_last, has_selector;
  int64_t waiting;  // absent states: the 'for' time (ms), else -1
  std::vector<std::vector<Insn>> filters;
};
struct IQuery {
  int type, partition;
  int64_t within;
  std::vector<IState> st;
};
struct IProgram {
  std::vector<std::vector<int>> stream_types;
  std::vector<IQuery> q;
};

struct WordReader {
  const int64_t* w;
  size_t n, i = 0;
  int64_t next() {
    if (i >= n) throw Error(SDH_E_INVALID, "IR blob truncated");
    return w[i++];
  }
};

std::vector<Insn> read_code(WordReader& r) {
  std::vector<Insn> c((size_t)r.next());
  for (auto& x : c) {
    int64_t w0 = r.next();
    x.op = (int)(w0 & 0xff);
    x.lt = (int)((w0 >> 8) & 0xff);
    x.rt = (int)((w0 >> 16) & 0xff);
    x.res = (int)((w0 >> 24) & 0xff);
    x.a = r.next();
    x.b = r.next();
    x.imm = r.next();
  }
  return c;
}

IProgram read_ir(const void* blob, size_t len) {
  if (!blob || len < 16 || memcmp(blob, "SDHIR001", 8) != 0) throw Error(SDH_E_INVALID, "bad IR magic");
  WordReader r{reinterpret_cast<const int64_t*>(static_cast<const char*>(blob) + 8), (len - 8) / 8};
  IProgram p;
  if (r.next() != 2) throw Error(SDH_E_INVALID, "unsupported IR version");
  p.stream_types.resize((size_t)r.next());
  for (auto& s : p.stream_types) {
    s.resize((size_t)r.next());
    for (auto& t : s) t = (int)r.next();
  }
  int64_t ns = r.next();
  for (int64_t k = 0; k < ns; ++k) {
    int64_t nb = r.next();
    for (int64_t j = 0; j < (nb + 7) / 8; ++j) r.next();
  }
  p.q.resize((size_t)r.next());
  for (auto& q : p.q) {
    q.type = (int)r.next();
    q.within = r.next();
    q.st.resize((size_t)r.next());
    q.partition = (int)r.next();
    r.next();
    for (auto& s : q.st) {
      s.kind = (int)r.next(); s.stream = (int)r.next(); s.is_start = (int)r.next();
      s.min = (int)r.next(); s.max = (int)r.next(); s.ltype = (int)r.next();
      s.partner = (int)r.next(); s.next_pre = (int)r.next(); s.next_every = (int)r.next();
      s.within_every = (int)r.next(); s.callback = (int)r.next(); s.this_last = (int)r.next();
      s.has_selector = (int)r.next();
      s.waiting = r.next();
      s.filters.resize((size_t)r.next());
      for (auto& f : s.filters) f = read_code(r);
    }
    int64_t n = r.next();
    for (int64_t k = 0; k < n; ++k) r.next();           // start ids
    n = r.next();
    for (int64_t k = 0; k < n; ++k) {                    // receivers
      r.next(); r.next();
      int64_t np = r.next();
      for (int64_t j = 0; j < np; ++j) r.next();
    }
    n = r.next();
    for (int64_t k = 0; k < n * 4; ++k) r.next();        // runtime tree
    n = r.next();
    for (int64_t k = 0; k < n; ++k) read_code(r);        // selector outputs (host-side projection)
  }
  return p;  // partitions follow; partitioned queries are rejected by the lowering below
}

// ------------------------------------------------------------------------------------------
// lowering: IR query -> ChainQuery (predicate atoms + captures)
// ------------------------------------------------------------------------------------------
// Compare domain of a typed compare (restates ExpressionParser.java:539-1220 + compare/**):
// ordering compares promote like Java binary numeric promotion; ==/!= of Long x Float compare in
// double (EqualCompareConditionExpressionExecutorLongFloat.java:36, ...FloatLong.java:37).
int domain_of(int lt, int rt, int op) {
  if (lt == T_STRING || lt == T_BOOL) return D_RAW;
  if (lt == T_DOUBLE || rt == T_DOUBLE) return D_F64;
  if (lt == T_FLOAT || rt == T_FLOAT) {
    if ((op == CMP_EQ || op == CMP_NE) && (lt == T_LONG || rt == T_LONG)) return D_F64;
    return D_F32;
  }
  if (lt == T_LONG || rt == T_LONG) return D_I64;
  return D_I32;
}

// conversion of an operand of attribute type t into the key of domain d (enum Conv)
int conv_of(int t, int d) {
  switch (d) {
    case D_I32:
    case D_I64: return t == T_INT ? CV_I64_INT : CV_I64_LONG;
    case D_F32: return t == T_INT ? CV_F32_INT : t == T_LONG ? CV_F32_LONG : CV_F64_FLOAT;  // float->double is exact
    case D_F64:
      return t == T_INT ? CV_F64_INT : t == T_LONG ? CV_F64_LONG : t == T_FLOAT ? CV_F64_FLOAT : CV_F64_DOUBLE;
    default: return CV_RAW;
  }
}

int64_t host_key(int64_t raw, int conv) {  // host twin of to_key() in nfa_chain.hip
  auto dbits = [](double d) { int64_t b; memcpy(&b, &d, 8); return b; };
  auto f_of = [](int64_t r) { uint32_t u = (uint32_t)r; float f; memcpy(&f, &u, 4); return f; };
  switch (conv) {
    case CV_I64_INT: return (int64_t)(int32_t)(uint32_t)raw;
    case CV_I64_LONG: return raw;
    case CV_F32_INT: return dbits((double)(float)(int32_t)(uint32_t)raw);
    case CV_F32_LONG: return dbits((double)(float)raw);
    case CV_F32_FLOAT:
    case CV_F64_FLOAT: return dbits((double)f_of(raw));
    case CV_F64_INT: return dbits((double)(int32_t)(uint32_t)raw);
    case CV_F64_LONG: return dbits((double)raw);
    default: return raw;
  }
}

int mask_of(int op) {
  switch (op) {
    case CMP_EQ: return CM_EQ;
    case CMP_NE: return CM_EQ | CM_NOT;
    case CMP_GT: return CM_GT;
    case CMP_GE: return CM_GT | CM_EQ;
    case CMP_LT: return CM_LT;
    default: return CM_LT | CM_EQ;
  }
}

struct Node {
  int kind;  // 0 leaf operand, 1 cmp, 2 and, 3 other
  Insn ins;
  int l = -1, r = -1;
};

struct Lowered {
  bool ok = false;
  std::string why;
  ChainQuery cq{};
  std::vector<int> streams;
};

Lowered lower_query(const IProgram& P, int qi) {
  Lowered L;
  const IQuery& q = P.q[qi];
  const int n = (int)q.st.size();
  auto fail = [&](const std::string& w) { L.ok = false; L.why = fmt("query %d: %s", qi, w.c_str()); return L; };
  if (q.partition >= 0) return fail("partitioned queries are not on the GPU path yet");
  if (q.type != Q_PATTERN) return fail("sequences are not on the GPU path yet");
  if (n < 1 || n > MAXS) return fail(fmt("%d states (chain kernel supports 1..%d)", n, MAXS));
  ChainQuery& c = L.cq;
  c.qid = qi;
  c.n_states = n;
  c.within = q.within;
  for (int s = 0; s < n; ++s) {
    const IState& st = q.st[s];
    if (st.kind != K_STREAM) return fail("count/logical states are not on the GPU path yet");
    if (st.is_start != (s == 0)) return fail("not a linear chain");
    if (st.next_pre != (s + 1 < n ? s + 1 : -1)) return fail("not a linear chain");
    if (s > 0 && st.next_every != -1) return fail("`every` inside the chain is not on the GPU path yet");
    if (s == 0 && st.next_every != -1 && st.next_every != 0) return fail("every scope");
    if (s > 0 && st.within_every != -1) return fail("within-every re-arm");
    if (st.callback != -1) return fail("count callback");
    if (st.has_selector != (s == n - 1)) return fail("selector placement");
    c.state_stream[s] = st.stream;
    if (std::find(L.streams.begin(), L.streams.end(), st.stream) == L.streams.end())
      L.streams.push_back(st.stream);
  }
  c.every = q.st[0].next_every == 0;
  for (int s = 0; s < n; ++s)
    if ((int)P.stream_types[q.st[s].stream].size() > MAXATTR) return fail("too many attributes");
  // a single input stream and `every` make event-chunk warm-up exact
  c.chunkable = (L.streams.size() == 1) && c.every && q.within >= 0 && n >= 2;

  int na = 0;
  for (int s = 0; s < n; ++s) {
    c.atom_begin[s] = na;
    std::vector<Atom> const_atoms, x_atoms;
    std::vector<int> x_cols;
    for (const auto& code : q.st[s].filters) {
      // postfix -> tree
      std::vector<Node> nodes;
      std::vector<int> stk;
      for (const Insn& ins : code) {
        Node nd;
        nd.ins = ins;
        if (ins.op == OP_CONST || ins.op == OP_ATTR) {
          nd.kind = 0;
        } else if (ins.op == OP_CMP || ins.op == OP_AND) {
          nd.kind = ins.op == OP_CMP ? 1 : 2;
          nd.r = stk.back(); stk.pop_back();
          nd.l = stk.back(); stk.pop_back();
        } else {
          return fail("filter uses or/not/is-null/arithmetic (general predicate kernel pending)");
        }
        nodes.push_back(nd);
        stk.push_back((int)nodes.size() - 1);
      }
      if (stk.size() != 1) return fail("malformed filter bytecode");
      // flatten the conjunction into atoms
      std::vector<int> todo{stk.back()};
      std::vector<int> leaves;
      while (!todo.empty()) {
        int x = todo.back(); todo.pop_back();
        if (nodes[x].kind == 2) { todo.push_back(nodes[x].r); todo.push_back(nodes[x].l); }
        else leaves.push_back(x);
      }
      for (int x : leaves) {
        Atom A{};
        const Node& nd = nodes[x];
        Insn li, ri;
        int op;
        if (nd.kind == 1) {
          if (nodes[nd.l].kind != 0 || nodes[nd.r].kind != 0)
            return fail("compare of computed values (general predicate kernel pending)");
          li = nodes[nd.l].ins;
          ri = nodes[nd.r].ins;
          op = (int)nd.ins.imm;
        } else if (nd.kind == 0 && nd.ins.res == T_BOOL) {
          // bare bool operand as a filter: FilterProcessor drops null and false
          li = nd.ins;
          ri = Insn{OP_CONST, 0, 0, T_BOOL, 0, 0, 1};
          op = CMP_EQ;
        } else {
          return fail("unsupported filter form");
        }
        const int dom = domain_of(li.res, ri.res, op);
        A.mask = mask_of(op);
        A.f64 = (dom == D_F32 || dom == D_F64) ? 1 : 0;
        // operand -> (kind, index, const key); single-event slots resolve only chain index
        // CURRENT (-1) and 0 (StateEvent.getStreamEvent:138-182), others read null
        auto operand = [&](const Insn& in, int& k, int& idx, int64_t& cst) -> bool {
          const int cv = conv_of(in.res, dom);
          idx = 0;
          cst = 0;
          if (in.op == OP_CONST) { k = OPK_CONST; cst = host_key(in.imm, cv); return true; }
          if (in.b != -1 && in.b != 0) { k = OPK_NULL; return true; }
          if (in.a > s) return false;
          const int st_stream = q.st[in.a].stream;
          int col = -1;
          for (int cc = 0; cc < c.n_col; ++cc)
            if (c.col_attr[cc] == in.imm && c.col_conv[cc] == cv && c.col_stream[cc] == st_stream) col = cc;
          if (col < 0) {
            if (c.n_col >= MAXCOL) return false;
            col = c.n_col++;
            c.col_attr[col] = (int)in.imm;
            c.col_conv[col] = cv;
            c.col_stream[col] = st_stream;
          }
          if (in.a == s) { k = OPK_CUR; idx = col; return true; }
          for (int cc = 0; cc < c.n_cap; ++cc)
            if (c.cap_slot[cc] == in.a && c.cap_col[cc] == col) { k = OPK_CAP; idx = cc; return true; }
          if (c.n_cap >= MAXCAP) return false;
          c.cap_slot[c.n_cap] = (int)in.a;
          c.cap_col[c.n_cap] = col;
          k = OPK_CAP;
          idx = c.n_cap++;
          return true;
        };
        if (!operand(li, A.lk, A.li, A.lc) || !operand(ri, A.rk, A.ri, A.rc))
          return fail("operand not addressable (too many columns / captures)");
        if (A.lk == OPK_CAP || A.rk == OPK_CAP) {
          x_atoms.push_back(A);
          x_cols.push_back(A.lk == OPK_CUR ? A.li : A.rk == OPK_CUR ? A.ri : -1);
        } else {
          const_atoms.push_back(A);
        }
      }
    }
    // partial-independent atoms first (tile-vectorized), capture readers last (per partial)
    if (na + (int)(const_atoms.size() + x_atoms.size()) > MAXATOM) return fail("too many predicate atoms");
    if (c.n_xa + (int)x_atoms.size() > MAXXA) return fail("too many capture-reading predicate atoms");
    for (const Atom& A : const_atoms) c.atoms[na++] = A;
    c.xa_first[s] = c.n_xa;
    c.xa_count[s] = (int)x_atoms.size();
    for (size_t k = 0; k < x_atoms.size(); ++k) {
      c.atoms[na] = x_atoms[k];
      c.xa_atom[c.n_xa] = na;
      c.xa_col[c.n_xa] = x_cols[k];
      ++c.n_xa;
      ++na;
    }
  }
  c.atom_begin[n] = na;
  for (int s = n + 1; s <= MAXS; ++s) c.atom_begin[s] = na;
  L.ok = true;
  return L;
}

int attr_width(int t) {
  switch (t) {
    case T_INT: case T_FLOAT: case T_STRING: return 4;
    case T_BOOL: return 1;
    default: return 8;
  }
}

// ------------------------------------------------------------------------------------------
// K_ratchet plan selection: 2-state `every e1=S[f0] -> e2=S[cur.a OP e1.a]`
// ------------------------------------------------------------------------------------------
struct RatchetPlan {
  bool ok = false;
  int stream = 0, key_attr = 0, key_conv = 0, key_kind = 0, xmask = 0;
  std::vector<RatchetAtom> f0;
  std::vector<int64_t> f0c;
  // K_gate (nfa_gate.hip): e2's event-only conjuncts `cur.b OP const` (empty: plain K_ratchet)
  std::vector<RatchetAtom> g;
  std::vector<int64_t> gc;
  int64_t within = -1;
  // grouping signature: everything except the per-lane constants and `within`
  std::vector<int64_t> sig() const {
    std::vector<int64_t> v{stream, key_kind, key_attr, key_conv, xmask, within >= 0, (int64_t)f0.size(),
                           (int64_t)g.size()};
    for (const auto* atoms : {&f0, &g})
      for (const auto& a : *atoms)
        v.insert(v.end(), {a.attr, a.conv, a.cur_left, a.mask, a.f64, a.cur2, a.attr2, a.conv2});
    return v;
  }
};

// an event-only atom `cur OP const` / `const OP cur` (a start filter's or a gate's) as a RatchetAtom
// and its constant; false for any other operand shape
bool const_atom(const ChainQuery& c, const Atom& A, RatchetAtom& ra, int64_t& cst) {
  ra = RatchetAtom{};
  ra.mask = A.mask;
  ra.f64 = A.f64;
  if (A.lk == OPK_CUR && A.rk == OPK_CONST) {
    ra.attr = c.col_attr[A.li]; ra.conv = c.col_conv[A.li]; ra.cur_left = 1; cst = A.rc;
  } else if (A.lk == OPK_CONST && A.rk == OPK_CUR) {
    ra.attr = c.col_attr[A.ri]; ra.conv = c.col_conv[A.ri]; ra.cur_left = 0; cst = A.lc;
  } else {
    return false;
  }
  return true;
}

RatchetPlan ratchet_plan(const ChainQuery& c) {
  RatchetPlan r;
  if (c.n_states != 2 || !c.every || c.state_stream[0] != c.state_stream[1]) return r;
  if (c.n_cap != 1 || c.cap_slot[0] != 0) return r;
  if (c.xa_count[1] != 1 || c.xa_count[0] != 0) return r;
  const int x_at = c.xa_atom[c.xa_first[1]];
  // state 1's other atoms: event-only constant compares gate it (K_gate); none for K_ratchet
  for (int a = c.atom_begin[1]; a < c.atom_begin[2]; ++a) {
    if (a == x_at) continue;
    RatchetAtom ga;
    int64_t cst = 0;
    if (!const_atom(c, c.atoms[a], ga, cst) || r.g.size() >= (size_t)RMAXF0) return RatchetPlan();
    r.g.push_back(ga);
    r.gc.push_back(cst);
  }
  const Atom& X = c.atoms[x_at];
  int mask = X.mask;
  if (mask & CM_NOT) return r;
  if (!(mask & (CM_LT | CM_GT)) || ((mask & CM_LT) && (mask & CM_GT))) return r;  // ordering only
  int cur_col;
  if (X.lk == OPK_CUR && X.rk == OPK_CAP) {
    cur_col = X.li;
  } else if (X.lk == OPK_CAP && X.rk == OPK_CUR) {
    cur_col = X.ri;
    const int lt = mask & CM_LT, gt = mask & CM_GT;
    mask = (mask & CM_EQ) | (lt ? CM_GT : 0) | (gt ? CM_LT : 0);  // key OP cur == cur OP' key
  } else {
    return r;
  }
  if (c.cap_col[0] != cur_col) return r;  // key = e1 value of the same column and conversion
  const int conv = c.col_conv[cur_col];
  // both operands are the same column with the same conversion: a float column compared in
  // binary64 orders exactly as in binary32, an int column as int32 (32-bit ring entries)
  switch (conv) {
    case CV_F32_INT: case CV_F32_LONG: case CV_F32_FLOAT: case CV_F64_FLOAT: r.key_kind = KK_F32; break;
    case CV_I64_INT: case CV_F64_INT: r.key_kind = KK_I32; break;
    case CV_I64_LONG: r.key_kind = KK_I64; break;
    case CV_F64_LONG: case CV_F64_DOUBLE: r.key_kind = KK_F64; break;
    default: return r;
  }
  if (r.key_kind < 0) return r;
  if (!r.g.empty() && r.key_kind != KK_F32 && r.key_kind != KK_I32) return RatchetPlan();  // (K_gate: 32-bit keys)
  const int na0 = c.atom_begin[1] - c.atom_begin[0];
  if (na0 > RMAXF0) return r;
  for (int a = c.atom_begin[0]; a < c.atom_begin[1]; ++a) {
    const Atom& A = c.atoms[a];
    RatchetAtom ra{};
    ra.mask = A.mask;
    ra.f64 = A.f64;
    int64_t cst = 0;
    if (A.lk == OPK_CUR && A.rk == OPK_CONST) {
      ra.attr = c.col_attr[A.li]; ra.conv = c.col_conv[A.li]; ra.cur_left = 1; cst = A.rc;
    } else if (A.lk == OPK_CONST && A.rk == OPK_CUR) {
      ra.attr = c.col_attr[A.ri]; ra.conv = c.col_conv[A.ri]; ra.cur_left = 0; cst = A.lc;
    } else if (A.lk == OPK_CUR && A.rk == OPK_CUR && r.g.empty()) {  // (K_gate: constant atoms only)
      ra.attr = c.col_attr[A.li]; ra.conv = c.col_conv[A.li]; ra.cur_left = 1;
      ra.cur2 = 1; ra.attr2 = c.col_attr[A.ri]; ra.conv2 = c.col_conv[A.ri];
    } else {
      return r;  // null operands / constant-only atoms: leave them to K_chain
    }
    r.f0.push_back(ra);
    r.f0c.push_back(cst);
  }
  r.stream = c.state_stream[0];
  r.key_attr = c.col_attr[cur_col];
  r.key_conv = conv;
  r.xmask = mask;
  r.within = c.within;
  r.ok = true;
  return r;
}

// SDH_ALLOC_TRACE=1: one stderr line per device buffer (re)allocation (p99 push/poll latency hunts)
inline void alloc_trace(const char* what, size_t bytes) {
  const bool on = sdh::knob("SDH_ALLOC_TRACE") != nullptr;
  if (on) fprintf(stderr, "[sdh] alloc %s %zu bytes\n", what, bytes);
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  // grows by at least half its size (a buffer sized per push or per poll would otherwise be freed and
  // allocated again whenever the count edges up: hipFree synchronises the device, a p99 spike)
  // The first allocation takes an eighth more than asked: a buffer sized exactly by its first push
  // or poll reallocated at the next one a few elements larger (C2's 64K-push leg: a 1.1-s poll, eight
  // ~4-GB hipFree + hipMalloc pairs)
  void ensure(size_t want) {
    if (want <= n) return;
    const size_t cap = std::max(want + want / 8, n + n / 2);
    alloc_trace("ensure", cap * sizeof(T));
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, cap * sizeof(T)) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      HIPCHK(hipMalloc(&p, want * sizeof(T)));
      n = want;
      return;
    }
    n = cap;
  }
  // grow to at least `want` elements keeping the first `keep` (stream-ordered copy)
  void grow_keep(size_t want, size_t keep, hipStream_t s) {
    if (want <= n) return;
    // (an eighth more on the first allocation, as ensure; and at least 1 MB: growing state tables of a
    // few hundred KB doubled inside small pushes -- C2's 1-event pushes, a 1.1-ms p99)
    size_t cap = std::max(std::max(want + want / 8, n * 2), ((size_t)1 << 20) / sizeof(T));
    alloc_trace("grow_keep", cap * sizeof(T));
    T* q = nullptr;
    if (hipMalloc(&q, cap * sizeof(T)) != hipSuccess) {
      (void)hipGetLastError();
      cap = want;
      if (hipMalloc(&q, cap * sizeof(T)) != hipSuccess)
        throw Error(SDH_E_CAPACITY, fmt("device memory exhausted growing a %zu-byte buffer", cap * sizeof(T)));
    }
    if (p && keep) HIPCHK(hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    if (p) HIPCHK(hipFree(p));
    p = q;
    n = cap;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

// host output buffer of a poll: pinned when the runtime grants it (faster D2H), else pageable
template <class T>
struct HostBuf {
  T* p = nullptr;
  size_t n = 0;
  bool pinned = false;
  void ensure(size_t want) {
    if (want <= n) return;
    release();
    const size_t cap = std::max(want + want / 8, n * 2);  // (an eighth of headroom, as DevBuf)
    alloc_trace("host", cap * sizeof(T));
    if (hipHostMalloc((void**)&p, cap * sizeof(T), hipHostMallocDefault) == hipSuccess) {
      pinned = true;
    } else {
      (void)hipGetLastError();
      p = (T*)malloc(cap * sizeof(T));
      if (!p) throw Error(SDH_E_CAPACITY, "host memory exhausted for the poll output");
      pinned = false;
    }
    n = cap;
  }
  void release() {
    if (!p) return;
    if (pinned) (void)hipHostFree(p);
    else free(p);
    p = nullptr;
  }
  ~HostBuf() { release(); }
};


}  // namespace

struct sdh_engine {
  sdh_config cfg{};
  int dev = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  IProgram prog;
  std::vector<Lowered> lq;           // local (this shard's) queries
  int K = 1, pcap = 64, rec_words = 3;
  DevBuf<ChainQuery> d_q;
  DevBuf<InstHeader> d_hdr[2];
  DevBuf<int64_t> d_part[2];
  std::vector<int> cur;              // which buffer holds each local query's state
  // batch staging for host-resident input
  DevBuf<uint8_t> d_batch;           // a host batch's columns in HBM (stage_host_batch)
  HostBuf<uint8_t> stage[2];         // pinned staging slots
  hipEvent_t ev_stage[2] = {nullptr, nullptr}, ev_h0 = nullptr, ev_h1 = nullptr;
  int stage_next = 0;
  hipStream_t h2d = nullptr;         // side stream of host-to-device batch copies
  std::vector<int64_t> prev_ts;      // per stream
  int64_t seq = 0;
  // last launch
  DevBuf<WorkItem> d_work;
  DevBuf<int64_t> d_seg_count, d_seg_off, d_dst_off, d_match;
  DevBuf<int32_t> d_err;
  std::vector<WorkItem> work;
  std::vector<int64_t> seg_count;
  int64_t device_matches = 0;        // K_chain matches of the last push
  // device match table (matches.hip): every match since the last poll with its R18 sort keys
  struct Table {
    DevBuf<uint64_t> hi, lo[MAXLO];
    DevBuf<int64_t> seq, q, key, ts, woff, wlen, words;
    int64_t n = 0, nw = 0;           // rows / words used
    int n_lo = 0;                    // tiebreak passes the rows need
    bool placed = false;             // the rows are K_ratchet matches already in R18 order in po_*
    // chunk delivery keys (nfa_types.h): allocated once a chunk push joins the window; rows
    // [0, ck_n) have theirs, the rest are single-event rows filled at the poll
    DevBuf<uint64_t> chi, clo;
    bool chunked = false;
    bool chunk_pushed = false;       // a chunk push joined the window (every rank alike: same pushes)
    int64_t ck_n = 0;
    int64_t max_run = 0;             // largest run start / key position a chunk row carries
  } mt;
  // the chunk push in progress (sdh_batch.chunk): its first event's seq, its length, and per
  // partition keyed on its stream each event's same-key run start (ck_runs[slot][event])
  struct Chunk {
    bool active = false;
    int64_t first_seq = 0, n = 0;
    int stream = -1;
  } ck;
  DevBuf<int32_t> ck_runs, d_ck_major, d_ck_minor, d_ck_qslot;
  std::vector<int32_t> ck_major, ck_minor;  // [query][stream] subscriber rank (+1), rank in partition
  int64_t seq_ref = 0;               // global seq at the last poll (<= every trigger seq in mt)
  DevBuf<int32_t> d_out_rank;        // [query][stream] R18 receiver rank
  DevBuf<int32_t> d_qinfo;           // [query] (states, stream of the last state)
  // poll scratch and outputs (device), host copies of the outputs
  DevBuf<uint64_t> p_keys;
  DevBuf<int32_t> p_perm;
  DevBuf<uint8_t> p_temp;
  DevBuf<int64_t> po_q, po_key, po_ts, po_seq, po_tb, po_len, po_off, po_words;
  HostBuf<int64_t> ho_q, ho_key, ho_ts, ho_seq, ho_tb, ho_off, ho_words;
  // compact rows (sdh_matches_compact): a placed window's rows live here (the ABI columns are
  // filled from them at a full poll), with the window's event times ts_log[seq - seq_ref]; cw =
  // 2 + the most states any query has
  DevBuf<int32_t> pc_rows, pc_err;
  DevBuf<int64_t> ts_log;
  HostBuf<int32_t> hc_rows;
  int cw = 4;
  // ---- K_gen (general interpreter) ----
  kg::LProgram lp;                   // full IR (receivers, runtime tree, partitions)
  std::vector<int> out_rank;         // R18 rank per (query, stream)
  std::vector<kg::GQuery> gq;
  DevBuf<kg::GQuery> d_gq;
  std::vector<int32_t> lane_q;       // [group][64]
  DevBuf<int32_t> d_lane_q;
  DevBuf<int64_t> d_lconst;          // [group][lc_slots][64] lane constants (kg::LaneConsts)
  int lc_slots = kg::LC_FIRST;
  std::vector<int32_t> group_tmpl;   // [group] shape template (a member query)
  DevBuf<int32_t> d_group_tmpl;
  std::vector<int32_t> group_seq;    // [group] window length S when the group runs on K_seq, else 0
  std::map<int, hipFunction_t> seq_spec;  // K_seq shape template -> its shape-compiled kernel (spec.h)
  std::vector<DevBuf<int32_t>> d_glists;  // [stream] unpartitioned groups: K_seq rows, then K_gen groups
  std::vector<DevBuf<int64_t>> seq_tail;  // [stream] last SEQ_TMAX events (K_seq windows)
  std::vector<int32_t> seq_tail_len;
  int gB32 = 1, gB64 = 1;
  int gHotS = 1, gHotNU = 1;  // K_gen LDS hot-word cache extents (max states / node-mask words)
  kg::Sizing gsz;                    // K_gen pool sizing (grows on overflow: gen_relayout)
  // absent states (kgen.h fire_timers): the runtime's start time and whether any query has them
  bool started = false;
  int64_t start_ts = 0;
  bool has_absent = false;
  bool has_fanout = false;           // a partition query reads a stream the partition does not key
  DevBuf<int32_t> d_fan_rank;        // [query][stream] its rank within the partition (fan-out), -1
  int64_t advance_to = INT64_MIN;    // set while a time advance runs (sdh_engine_advance_time)
  std::vector<char> gq_arena;        // [gq] the query runs on K_gen (has an instance arena)
  int64_t gen_regrows = 0;           // pool growths so far (sdh_stats)
  struct GenSet {
    int partition = -1;              // -1: the unpartitioned K_gen queries
    int group_base = 0, n_groups = 0;
    int64_t key_cap = 0;             // instance blocks = key_cap * n_groups (partitioned)
    DevBuf<int32_t> a32;
    DevBuf<int64_t> a64;
    DevBuf<int32_t> s32;             // scratch arenas of event chunks 1.. (unpartitioned sets)
    DevBuf<int64_t> s64;
    // exact re-runs: the blocks the current pass modifies, as they were before it (gen_journal)
    DevBuf<int32_t> j32;
    DevBuf<int64_t> j64, jidx;
    int64_t jn = 0;
  };
  std::vector<std::unique_ptr<GenSet>> gsets;
  // per partition: PartitionRuntime's key -> instance map (dense key ids), shared by the
  // partition's K_gen set and K_part sets (PartitionRuntime.java:257-306)
  struct Route {
    DevBuf<unsigned long long> tkey;
    DevBuf<int32_t> tid, n_keys;
    DevBuf<int64_t> key_of_id;
    int64_t tmask = 0, max_keys = 0;
    // fan-out partitions: keys in creation order (dense id, value), for the junction-map order
    bool track = false;
    int kkind = 0;                   // key values: 0 int / long, 1 bool, 2 string (dictionary ids),
                                     // 3 float, 4 double (raw bits; NaN canonical)
    int64_t nk_seen = 0;
    std::vector<int64_t> korder_kid, korder_key;
    DevBuf<int64_t> nk_tmp;
    struct Fan {
      int64_t n = -1;  // keys the positions cover
      DevBuf<int32_t> pos;
    };
    std::map<int, Fan> fan;  // [stream] per-kid positions in that stream's junction map
  };
  std::vector<std::unique_ptr<Route>> routes;  // [partition] (null: no device set uses it)
  // K_part (nfa_part.hip): one set per (partition, kind); state blocks (key, group) double-buffered
  // per key: cur[kid] says which of st[0] / st[1] holds the key's current tables
  struct PartSet {
    int partition = -1, kind = 0;
    int group_base = 0, n_groups = 0;
    int cap = 8, ew = 3, sA = 1, sB = 2, cmax = 0, n_e1 = 0, n_first = 0, n_last = 0;
    int64_t key_cap = 0;
    bool ran = false;                // launched in the current pass
    DevBuf<int64_t> st;              // [2][key_cap * n_groups][PK_HDR + cap * ew][64]
    DevBuf<int32_t> cur, nxt;        // [key_cap]
    int64_t bw() const { return PK_HDR + (int64_t)cap * ew; }
    std::map<int, hipFunction_t> spec;  // shape template -> shape-compiled kernel (spec.h)
  };
  std::vector<std::unique_ptr<PartSet>> psets;
  // K_slab (nfa_slab.hip): one set per partition; its queries' partials as sparse entries, one block
  // per (key, group) in nsub sub-rings of a slab, found through the directory [key][group]
  struct SlabSet {
    int partition = -1;
    int group_base = 0, n_groups = 0;
    int64_t key_cap = 0;
    std::vector<slab::Shape> shapes;
    std::vector<int32_t> group_shape, group_ew;
    DevBuf<slab::Shape> d_shapes;
    DevBuf<int32_t> d_group_shape, d_group_ew;
    std::vector<std::vector<int32_t>> glist;  // [stream] set groups reading it
    std::vector<DevBuf<int32_t>> d_glist;
    DevBuf<uint64_t> dir;                     // [key_cap * n_groups]
    int nsub = 256;                           // sub-rings (separate buffers: they grow one at a time)
    std::vector<uint32_t*> ring;
    std::vector<int64_t> cap;                 // words per ring
    DevBuf<uint32_t*> d_ring;
    DevBuf<int64_t> d_cap;
    DevBuf<unsigned long long> head, tail, head_bak;
    std::vector<unsigned long long> h_head, h_tail, h_push0;  // h_push0: heads before the last push
    // Ring buffers are carved from an arena of large chunks that are never returned while the engine
    // lives: a ring that grows takes a new range and gives its old one back to the free list (adjacent
    // free ranges merge), so growing costs no driver allocation once the arena holds enough. (A
    // hipMalloc of GBs stalls for seconds from time to time on this driver, whether or not memory
    // was freed; tools/alloc_probe.py.) sdh_engine_reserve sizes the arena up front.
    struct Chunk {
      uint8_t* base;
      size_t bytes;
      std::map<size_t, size_t> free;  // offset -> length
    };
    std::vector<Chunk> chunks;
    size_t arena_bytes = 0;
    bool add_chunk(size_t bytes) {
      void* p = nullptr;
      alloc_trace("slab_chunk", bytes);
      if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
      }
      chunks.push_back(Chunk{(uint8_t*)p, bytes, {}});
      chunks.back().free[0] = bytes;
      arena_bytes += bytes;
      return true;
    }
    uint32_t* take(size_t bytes) {
      for (auto& c : chunks)
        for (auto it = c.free.begin(); it != c.free.end(); ++it) {
          if (it->second < bytes) continue;
          const size_t off = it->first, len = it->second;
          c.free.erase(it);
          if (len > bytes) c.free[off + bytes] = len - bytes;
          return (uint32_t*)(c.base + off);
        }
      return nullptr;
    }
    uint32_t* alloc_ring(int64_t words) {
      const size_t bytes = ((size_t)words * 4 + 4095) & ~(size_t)4095;
      if (uint32_t* p = take(bytes)) return p;
      // a new chunk: as large as the arena so far (the chunks double), or what the device still has
      size_t want = std::max(bytes, std::max(arena_bytes, (size_t)1 << 30));
      for (;;) {
        if (add_chunk(want)) return take(bytes);
        if (want == bytes) return nullptr;
        want = std::max(bytes, want / 2);
      }
    }
    void free_ring(uint32_t* p, int64_t words) {
      if (!p) return;
      const size_t bytes = ((size_t)words * 4 + 4095) & ~(size_t)4095;
      for (auto& c : chunks) {
        if ((uint8_t*)p < c.base || (uint8_t*)p >= c.base + c.bytes) continue;
        size_t off = (size_t)((uint8_t*)p - c.base), len = bytes;
        auto nx = c.free.lower_bound(off);
        if (nx != c.free.end() && nx->first == off + len) {
          len += nx->second;
          nx = c.free.erase(nx);
        }
        if (nx != c.free.begin()) {
          auto pv = std::prev(nx);
          if (pv->first + pv->second == off) {
            off = pv->first;
            len += pv->second;
            c.free.erase(pv);
          }
        }
        c.free[off] = len;
        return;
      }
    }
    ~SlabSet() {
      for (auto& c : chunks) (void)hipFree(c.base);
    }
    DevBuf<long long> live, live_bak;
    DevBuf<unsigned long long> traffic;       // block bytes read + written by the last launch
    DevBuf<uint64_t> journal, journal_idx;
    int64_t items = 0;                        // items of this pass's launch (0: not launched)
    int lds_words = 4096;                     // LDS rows (uint32 words) of the large tier
    DevBuf<int32_t> defer, defer_n;           // items deferred to the large tier (nfa_slab.hip)
    int64_t deferred = 0;
    int64_t cleanings = 0, growths = 0;
  };
  std::vector<std::unique_ptr<SlabSet>> ssets;
  DevBuf<int32_t> d_serr;            // per K_slab set: [0] LDS capacity, [1] slab space, [2] output overflow
  int64_t slab_items = 0;            // K_slab work items of the last push
  std::vector<int64_t> part_kept;    // per partition: events of the last push routed to a key here
  DevBuf<int32_t> d_perr;            // per K_part set: [0] entry capacity, [2] output overflow
  DevBuf<unsigned long long> d_pprof;  // SDH_PART_PROF measurement builds: phase clocks
  DevBuf<int64_t> r_key;
  DevBuf<int64_t> t_pm;              // indexed timer sweep: the batch's timestamp prefix max
  DevBuf<int32_t> t_kseg, t_flag;    // per known key its routed segment; ts-order flag
  DevBuf<uint8_t> t_temp;
  DevBuf<uint32_t> r_kid, r_kid_s, r_uniq;
  DevBuf<int32_t> r_idx, r_idx_s, r_cnt, r_off, r_nruns;
  DevBuf<uint8_t> r_temp;
  DevBuf<int64_t> g_out;
  int64_t g_out_cap = 0;             // K_gen match record words per push
  DevBuf<unsigned long long> g_out_next;
  DevBuf<unsigned long long> g_nrec;
  DevBuf<int64_t> g_rec_off;         // word offset of each K_gen / K_seq / K_part record of the last push
  DevBuf<int64_t> g_tw;              // their table words, scanned (append_gen)
  DevBuf<uint8_t> g_twtemp;
  DevBuf<unsigned long long> g_nwide;  // K_gen-format (not narrow) records of the last append
  // sdh_engine_poll_compact_ex outputs
  DevBuf<int64_t> px_cw, px_key, px_tb;
  DevBuf<int32_t> px_chain;
  DevBuf<uint8_t> px_temp;
  HostBuf<int64_t> hx_key, hx_tb;
  HostBuf<int32_t> hx_chain;
  DevBuf<const int64_t*> d_qkeys;    // [query] its partition's key table (narrow K_part records)
  DevBuf<uint8_t> sb_buf;            // a batch in key order (K_part reads; sdh_sort_batch)
  DevBuf<unsigned long long> g_rec_next;
  int64_t g_dev_matches = 0;         // K_gen / K_seq matches of the last push
  int64_t g_used = 0;                // words of the last push's records in g_out
  bool g_journal = false;            // the current K_gen pass journals the blocks it modifies
  // ---- K_ratchet groups ----
  std::vector<RatchetGroup> rg;
  std::vector<int> rcur;             // per group: buffer holding its deques
  DevBuf<RatchetGroup> d_rg;
  DevBuf<RatchetState> d_rst[2];
  DevBuf<int64_t> d_rts[2], d_rsq[2], d_rky[2];
  DevBuf<RatchetItem> d_ritems;
  std::vector<RatchetItem> ritems;
  DevBuf<int64_t> d_rmatch;
  DevBuf<int32_t> d_blk_count, d_blk_next, d_blk_group;
  DevBuf<int32_t> d_blk_side;            // K_ratchet rec4 blocks: side entries (-1: an 8- / 16-B block)
  int64_t r_rec4_reruns = 0;             // pushes re-run with 8-B records (a rec4 distance reached 2^26)
  DevBuf<unsigned long long> d_rtotal;  // device records: [0] entries, [2] bytes written
  int r_wide = 0;
  int64_t r_blocks = 0;              // capacity in blocks
  int r_blk_recs = 8192;
  int r_blocks_used = 0;             // of the last launch
  int64_t r_blk_taken = 0;           // blocks the last launch took
  double r_rec_bytes = 0;            // device records: bytes the last launch wrote (entries + side entries)
  int r_rec4 = 0;                    // device records: the last launch wrote rec4 blocks (SIM launches)
  DevBuf<int32_t> d_rlane_q;         // [group][64] query of each K_ratchet lane (-1 idle; sdh_records)
  DevBuf<int64_t> d_rrow_off;        // sdh_engine_records_compact: per-block row offsets
  DevBuf<uint8_t> d_rrow_tmp;
  bool dev_polled = false;           // the last push's device records were handed out
  int64_t last_n = 0, last_seq_base = 0;  // the last push's events and first seq
  // direct R18 placement (nfa_ratchet.hip PM): the (event, group cell) match counts, scanned
  DevBuf<int32_t> p_cnt;
  std::vector<int> place_cells;     // [stream] K_ratchet groups reading it (0: not placeable)
  // string dictionary ids -> (String.hashCode, UTF-16 length) of their text (sdh_engine_set_strings):
  // the fan-out order of partitions keyed by a string attribute
  std::unordered_map<int32_t, std::pair<int32_t, int64_t>> str_info;
  bool r_placing = false;            // the last K_ratchet launch placed its matches (compact rows)
  int64_t r_place_row0 = 0;          //   from this row of pc_rows
  DevBuf<uint8_t> p_ptemp;
  int64_t r_seq_base = 0;            // seq of the last launch's first event
  std::vector<int32_t> r_blk_count;
  int slab_lds_small = 1024;          // K_slab small-tier LDS rows (SDH_SLAB_LDS_SMALL)
  int xcd = 0;                       // per-XCD item ranges in the K_gen / K_seq / K_part / K_slab launches
                                     // (dev::grid_item; SDH_XCD=1: measured neutral)
  int rML = 8;                       // LDS ring entries per lane (power of two)
  double r_waves = 0;                // resident-wave target per launch (0: CUs x occupancy)
  int n_cu = 256;
  std::vector<std::array<int, 4>> r_sum_specs;  // tile-summary rows: (stream, attr, conv, key kind)
  DevBuf<uint64_t> d_tsmax, d_tsmin;
  DevBuf<uint8_t> d_tshas;
  int rSC = 256;                     // global spill ring entries per lane (power of two)
  int64_t rsmax = RSMAX;             // persisted deque entries per lane (grows with rSC)
  DevBuf<uint4> d_rspillA;
  DevBuf<int64_t> d_rlts;
  DevBuf<uint32_t> d_rspillB;
  std::vector<char> r_full_expiry;   // per stream: timestamps were seen out of order
  int64_t r_matches = 0;
  double r_kernel_ms = 0, r_kernel_bytes = 0;
  sdh_stats stats{};
  std::string err;
  std::string broken;                // set when a failed push left the state undefined
  std::vector<std::pair<std::string, std::string>> knobs;  // sdh_config.debug (knobs.h)
  // ---- multi-GPU exchange (comm.h; sdh_engine_push_bcast / sdh_engine_gather) ----
  sdh_comm* comm = nullptr;          // not owned
  DevBuf<uint8_t> x_batch;           // a broadcast batch received from the root
  DevBuf<uint64_t> x_keys;           // this rank's merge keys, one run
  // rank 0: every rank's run concatenated, and the merged output
  DevBuf<int64_t> xg_q, xg_key, xg_ts, xg_seq, xg_tb, xg_off, xg_words;
  DevBuf<uint64_t> xg_keys;
  DevBuf<int64_t> go_q, go_key, go_ts, go_seq, go_tb, go_len, go_off, go_src, go_pos, go_words;
  DevBuf<uint8_t> go_temp;
};

namespace {

void ensure_state(sdh_engine* e) {
  const size_t nq = e->lq.size();
  for (int b = 0; b < 2; ++b) {
    e->d_hdr[b].ensure(std::max<size_t>(nq, 1));
    e->d_part[b].ensure(std::max<size_t>(nq, 1) * NF * e->pcap);
  }
  // initial state: every query seeded (QueryRuntime.init -> StreamPreStateProcessor.init:157-166)
  std::vector<InstHeader> h(nq);
  for (auto& x : h) x = InstHeader{1, 0, 0, 0};
  std::vector<int64_t> part(nq * NF * e->pcap, 0);
  for (size_t q = 0; q < nq; ++q)
    for (int l = 0; l < e->pcap; ++l) part[(q * NF + F_STATE) * e->pcap + l] = -1;
  for (int b = 0; b < 2; ++b) {
    if (nq) {
      HIPCHK(hipMemcpy(e->d_hdr[b].p, h.data(), nq * sizeof(InstHeader), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_part[b].p, part.data(), part.size() * 8, hipMemcpyHostToDevice));
    }
  }
  e->cur.assign(nq, 0);
}

// ---- device match table (matches.hip) ----
sdh::MatchTable table_view(sdh_engine* e) {
  sdh::MatchTable T{};
  auto& t = e->mt;
  T.hi = t.hi.p;
  for (int k = 0; k < MAXLO; ++k) T.lo[k] = t.lo[k].p;
  T.seq = t.seq.p;
  T.q = t.q.p;
  T.key = t.key.p;
  T.ts = t.ts.p;
  T.woff = t.woff.p;
  T.wlen = t.wlen.p;
  T.words = t.words.p;
  T.chi = t.chi.p;
  T.clo = t.clo.p;
  return T;
}

// room for `rows` more rows and `words` more words (contents kept)
void table_reserve(sdh_engine* e, int64_t rows, int64_t words) {
  auto& t = e->mt;
  const size_t want = (size_t)(t.n + rows), keep = (size_t)t.n;
  t.hi.grow_keep(want, keep, e->stream);
  for (int k = 0; k < MAXLO; ++k) t.lo[k].grow_keep(want, keep, e->stream);
  t.seq.grow_keep(want, keep, e->stream);
  t.q.grow_keep(want, keep, e->stream);
  t.key.grow_keep(want, keep, e->stream);
  t.ts.grow_keep(want, keep, e->stream);
  t.woff.grow_keep(want, keep, e->stream);
  t.wlen.grow_keep(want, keep, e->stream);
  t.words.grow_keep((size_t)(t.nw + words), (size_t)t.nw, e->stream);
}

// the last push's K_chain matches (per work item output segments) -> table
void append_chain(sdh_engine* e) {
  const int n_items = (int)e->work.size();
  if (e->device_matches == 0 || n_items == 0) return;
  std::vector<int64_t> seg_off(n_items), dst_off(n_items);
  int64_t acc = 0;
  for (int i = 0; i < n_items; ++i) {
    seg_off[i] = e->work[i].seg_off;
    dst_off[i] = acc;
    acc += e->seg_count[i];
  }
  table_reserve(e, acc, acc * 2 * MAXS);
  e->d_seg_off.ensure(n_items);
  e->d_dst_off.ensure(n_items);
  HIPCHK(hipMemcpyAsync(e->d_seg_off.p, seg_off.data(), n_items * 8, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(e->d_dst_off.p, dst_off.data(), n_items * 8, hipMemcpyHostToDevice, e->stream));
  HIPCHK(sdh_append_chain(e->d_match.p, e->d_seg_off.p, e->d_seg_count.p, e->d_dst_off.p, e->rec_words, n_items,
                          e->d_qinfo.p, e->seq_ref, e->d_out_rank.p, (int)e->prog.stream_types.size(),
                          table_view(e), e->mt.n, e->mt.nw, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->mt.n += acc;
  e->mt.nw += acc * 2 * MAXS;
  e->mt.n_lo = std::max(e->mt.n_lo, e->rec_words - 3);
}

// the last push's K_ratchet match blocks -> table (ts_col: the batch's ts column, still valid)
void append_ratchet(sdh_engine* e, const int64_t* ts_col, int64_t seq_base) {
  const int nb = e->r_blocks_used;
  if (nb == 0 || e->r_matches == 0) return;
  std::vector<int64_t> dst_off(nb);
  int64_t acc = 0;
  for (int i = 0; i < nb; ++i) {
    dst_off[i] = acc;
    acc += e->r_blk_count[i];
  }
  table_reserve(e, acc, acc * 4);
  e->d_dst_off.ensure(nb);
  HIPCHK(hipMemcpyAsync(e->d_dst_off.p, dst_off.data(), nb * 8, hipMemcpyHostToDevice, e->stream));
  HIPCHK(sdh_append_ratchet(e->d_rmatch.p, e->r_blk_recs, e->r_wide, e->d_blk_count.p, e->d_blk_group.p,
                            e->d_dst_off.p, e->d_rg.p, ts_col, seq_base, e->seq_ref, e->d_out_rank.p,
                            (int)e->prog.stream_types.size(), nb, table_view(e), e->mt.n, e->mt.nw, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->mt.n += acc;
  e->mt.nw += acc * 4;
  e->mt.n_lo = std::max(e->mt.n_lo, 1);
}

// per query its partition's key table, on the device (narrow K_part records carry the key's dense id)
void upload_qkeys(sdh_engine* e) {
  const size_t nq = std::max<size_t>(1, e->prog.q.size());
  std::vector<const int64_t*> qk(nq, nullptr);
  for (const auto& g : e->gq)
    if (g.partition >= 0 && g.partition < (int)e->routes.size() && e->routes[g.partition] && g.qid >= 0 &&
        (size_t)g.qid < nq)
      qk[(size_t)g.qid] = e->routes[g.partition]->key_of_id.p;
  e->d_qkeys.ensure(nq);
  HIPCHK(hipMemcpyAsync(e->d_qkeys.p, qk.data(), nq * sizeof(void*), hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
}

// the last push's K_gen / K_seq / K_part records -> table: each record's table words (narrow K_part
// records expand), scanned, then the rows. bts / seq_base / stream: the push's batch (narrow records
// take their trigger's ts from it); null for a time advance (timer records only)
void append_gen(sdh_engine* e, const int64_t* bts, int64_t seq_base, int stream) {
  const int64_t n_rec = e->g_dev_matches;
  if (n_rec == 0) return;
  e->g_tw.ensure((size_t)n_rec + 1);
  e->g_twtemp.ensure(sdh_gen_words_temp_bytes(n_rec));
  e->g_nwide.ensure(1);
  HIPCHK(sdh_gen_words(e->g_out.p, e->g_rec_off.p, n_rec, e->g_tw.p, e->g_twtemp.p, e->g_twtemp.n, e->g_nwide.p,
                       e->stream));
  int64_t words = 0;
  unsigned long long n_wide = 0;
  HIPCHK(hipMemcpyAsync(&n_wide, e->g_nwide.p, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&words, e->g_tw.p + n_rec, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  table_reserve(e, n_rec, words);
  upload_qkeys(e);
  HIPCHK(sdh_append_gen(e->g_out.p, e->g_rec_off.p, n_rec, e->seq_ref, e->d_out_rank.p,
                        e->has_fanout ? e->d_fan_rank.p : nullptr, (int)e->prog.stream_types.size(), table_view(e),
                        e->mt.n, e->mt.nw, e->g_tw.p, bts, seq_base, stream, e->d_qkeys.p, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->mt.n += n_rec;
  e->mt.nw += words;
  // timer records: (key, query, time); fan-out records: (position, rank, emission). K_part's narrow
  // records need no tiebreak pass: the matches of one (trigger event, query) come from one lane,
  // which emits them in list order, so the stable sort on the primary key keeps them in it
  if (n_wide) e->mt.n_lo = std::max(e->mt.n_lo, e->has_absent || e->has_fanout ? 3 : 1);
}

void table_clear(sdh_engine* e) {
  e->mt.n = 0;
  e->mt.nw = 0;
  e->mt.n_lo = 0;
  e->mt.placed = false;
  e->mt.chunked = false;
  e->mt.chunk_pushed = false;
  e->mt.ck_n = 0;
  e->mt.max_run = 0;
  e->seq_ref = e->seq;
  e->r_placing = false;  // (the placed rows are gone)
}

// chunk keys of rows [ck_n, r1): single-event rows (chunk = false), or the rows the chunk push in
// progress appended (matches.hip chunk_keys_kernel)
void chunk_keys(sdh_engine* e, int64_t r1, bool chunk) {
  auto& t = e->mt;
  if (r1 <= t.ck_n) return;
  t.chi.grow_keep((size_t)r1, (size_t)t.ck_n, e->stream);
  t.clo.grow_keep((size_t)r1, (size_t)t.ck_n, e->stream);
  const int ns = (int)e->prog.stream_types.size();
  HIPCHK(sdh_chunk_keys(table_view(e), t.ck_n, r1, chunk ? 1 : 0, e->ck.first_seq - e->seq_ref, e->ck.first_seq,
                        e->ck.stream, ns, e->d_ck_major.p, e->d_ck_minor.p, e->d_ck_qslot.p, e->ck_runs.p, e->ck.n,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  t.ck_n = r1;
}

// the rows a sub-push of the chunk in progress appended, from row n0 on
void chunk_rows(sdh_engine* e, int64_t n0) {
  if (e->mt.n <= n0) return;
  e->mt.chunked = true;
  chunk_keys(e, n0, false);
  chunk_keys(e, e->mt.n, true);
}

// keys this push created (ids [nk_seen, new_n)), in the order of their first events: the order
// PartitionRuntime.clonePartition adds them to every receiver's junction map
void track_new_keys(sdh_engine* e, sdh_engine::Route& rt, int64_t new_n, int64_t nruns, int kkind) {
  const int64_t m = new_n - rt.nk_seen;
  rt.nk_tmp.ensure((size_t)(2 * m));
  HIPCHK(sdh_new_keys(e->r_uniq.p, e->r_nruns.p, nruns, e->r_off.p, e->r_idx_s.p, rt.key_of_id.p, rt.nk_seen, new_n,
                      rt.nk_tmp.p, e->stream));
  std::vector<int64_t> v((size_t)(2 * m));
  HIPCHK(hipMemcpyAsync(v.data(), rt.nk_tmp.p, v.size() * 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::vector<int64_t> ord((size_t)m);
  for (int64_t k = 0; k < m; ++k) ord[(size_t)k] = k;
  std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return v[(size_t)(2 * a)] < v[(size_t)(2 * b)]; });
  for (int64_t k : ord) {
    rt.korder_kid.push_back(rt.nk_seen + k);
    rt.korder_key.push_back(v[(size_t)(2 * k + 1)]);
  }
  rt.kkind = kkind;
  rt.nk_seen = new_n;
}

// per known key its position in the fan-out stream's junction map of "streamId + key" strings
// (chm_order.h), on the device; rebuilt when keys were added
const int32_t* fan_positions(sdh_engine* e, sdh_engine::Route& rt, const kg::LFanOut& fo, int64_t nk) {
  auto& f = rt.fan[fo.stream];
  if (f.n != nk) {
    const size_t m = std::min<size_t>((size_t)nk, rt.korder_key.size());
    std::vector<int32_t> hs(m), byk((size_t)std::max<int64_t>(1, nk), 0);
    for (size_t j = 0; j < m; ++j) {
      const int64_t k = rt.korder_key[j];
      if (rt.kkind == 2) {  // String.valueOf of a string is its text: its registered hash and length
        auto it = e->str_info.find((int32_t)k);
        if (it == e->str_info.end())
          throw Error(SDH_E_INVALID, fmt("partition key string id %lld has no text hash (sdh_engine_set_strings)", (long long)k));
        hs[j] = sdh::java_hash_cat_hashed(fo.id_hash, it->second.first, it->second.second);
      } else if (rt.kkind == 3 || rt.kkind == 4) {  // Float / Double.toString (java_fmt.h)
        hs[j] = sdh::java_hash_cat(fo.id_hash, rt.kkind == 3 ? sdh::jfmt::float_to_string((uint32_t)k)
                                                             : sdh::jfmt::double_to_string((uint64_t)k));
      } else {
        hs[j] = sdh::java_hash_cat(fo.id_hash, sdh::java_value_of(rt.kkind == 1, k));
      }
    }
    const std::vector<int32_t> pos = sdh::ChmOrder().positions(hs);
    for (size_t j = 0; j < m; ++j) byk[(size_t)rt.korder_kid[j]] = pos[j];
    f.pos.ensure(byk.size());
    HIPCHK(hipMemcpy(f.pos.p, byk.data(), byk.size() * 4, hipMemcpyHostToDevice));
    f.n = nk;
  }
  return f.pos.p;
}

// A push on a stream that fans out to every key of a string-keyed partition needs the text hash of
// every key it will reach (fan_positions). Checked before any kernel runs, so a missing
// sdh_engine_set_strings (e.g. after sdh_engine_restore) fails the push with SDH_E_INVALID and leaves
// the engine usable. (A push on the keyed stream creates keys but reaches no fan-out position.)
void check_fan_strings(const sdh_engine* e, int stream) {
  for (size_t pi = 0; pi < e->lp.parts.size() && pi < e->routes.size(); ++pi) {
    const sdh_engine::Route* rt = e->routes[pi].get();
    if (!rt || !rt->track || rt->kkind != 2 || !e->lp.parts[pi].fan(stream)) continue;
    for (int64_t k : rt->korder_key)
      if (e->str_info.find((int32_t)k) == e->str_info.end())
        throw Error(SDH_E_INVALID, fmt("partition key string id %lld has no text hash (sdh_engine_set_strings)", (long long)k));
  }
}

// A normal-mode push places its K_ratchet matches directly (nfa_ratchet.hip PM: COUNT per (event,
// group) cell, scan, WRITE as compact rows after the window's rows) when they are its only matches
// -- the chain and K_gen launches ran first and produced none, and the window holds no table rows
// --, the stream's groups are rank-ordered (place_cells), the cells stay within 2^30, the seqs of
// the window within 2^31 of seq_ref, and the launch runs without the full-expiry scan.
bool ratchet_placeable(const sdh_engine* e, int stream, int64_t seq_base, int64_t n_events, bool full) {
  const int nc = e->place_cells[(size_t)stream];
  return nc > 0 && !(e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) && !full && n_events > 0 && !e->ck.active &&
         e->device_matches == 0 && e->g_dev_matches == 0 && (e->mt.n == 0 || e->mt.placed) &&
         (double)n_events * nc < (double)(1 << 30) && seq_base + n_events - e->seq_ref < INT32_MAX &&
         !sdh::knob("SDH_NO_PLACE");
}

// a placed push joins the window: its rows are already in pc_rows; the compact rows carry seqs
// only, so the window keeps the pushed events' times (ts_log[seq - seq_ref])
void place_commit(sdh_engine* e, const int64_t* ts_col, int64_t seq_base, int64_t n_events) {
  e->mt.placed = true;
  if (e->r_matches == 0) return;  // (rows reference their own push's events only)
  const int64_t t0 = seq_base - e->seq_ref;
  e->ts_log.grow_keep((size_t)(t0 + n_events), (size_t)t0, e->stream);
  HIPCHK(hipMemcpyAsync(e->ts_log.p + t0, ts_col, (size_t)n_events * 8, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->mt.n += e->r_matches;
  ++e->stats.placed_pushes;
}

// placed rows -> general table rows (a later push of the window has other producers)
void placed_to_table(sdh_engine* e) {
  if (!e->mt.placed) return;
  const int64_t n = e->mt.n;
  e->mt.n = 0;
  e->mt.nw = 0;
  table_reserve(e, n, 4 * n);
  HIPCHK(sdh_placed_to_table(e->pc_rows.p, e->cw, n, e->ts_log.p, e->seq_ref, e->d_out_rank.p, e->d_qinfo.p,
                             (int)e->prog.stream_types.size(), table_view(e), e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->mt.n = n;
  e->mt.nw = 4 * n;
  e->mt.n_lo = std::max(e->mt.n_lo, 1);
  e->mt.placed = false;
}

int bits_of(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

// the ABI output arrays in HBM for n matches of tw words (po_*; off and len have n + 1 entries)
// (at least 64K rows: a window that edges past the last size would otherwise reallocate -- a
// device allocation inside the poll, the p99 of small pushes)
constexpr int64_t POLL_MIN_ROWS = 1 << 16;
void poll_reserve(sdh_engine* e, int64_t n, int64_t tw) {
  const size_t m = (size_t)std::max<int64_t>(n, POLL_MIN_ROWS);
  tw = std::max<int64_t>(tw, 4 * POLL_MIN_ROWS);
  n = std::max<int64_t>(n, POLL_MIN_ROWS);
  e->po_q.ensure(m);
  e->po_key.ensure(m);
  e->po_ts.ensure(m);
  e->po_seq.ensure(m);
  e->po_tb.ensure(m);
  e->po_len.ensure(n + 1);
  e->po_off.ensure(n + 1);
  e->po_words.ensure((size_t)std::max<int64_t>(tw, 1));
}

// R18 sort of the table's n > 0 rows and gather of the ABI arrays except the words; returns the
// sorted order (perm[i] = the table row of match i)
int32_t* table_order(sdh_engine* e, int64_t* total_words) {
  const int64_t n = e->mt.n;
  if (n >= INT32_MAX) throw Error(SDH_E_CAPACITY, "more than 2^31 matches between two polls");
  e->p_keys.ensure((size_t)n * 2);
  e->p_perm.ensure((size_t)n * 2);
  const size_t tb = sdh_poll_temp_bytes(n);
  e->p_temp.ensure(tb);
  poll_reserve(e, n, 0);
  // timer records' tiebreaks are a full timestamp, the query and the partition key
  const int lo_bits = e->has_absent ? 64 : std::max(1, bits_of((uint64_t)std::max<int64_t>(e->seq, 1 << 16)));
  const int hi_bits = bits_of((uint64_t)(e->seq - e->seq_ref)) + RANK_BITS;
  int clo_bits = 0;
  if (e->mt.chunked) {  // the window holds chunk rows: the single-event rows' chunk keys, 2 passes more
    chunk_keys(e, n, false);
    clo_bits = bits_of((uint64_t)e->mt.max_run) + RANK_BITS;
  }
  int32_t* perm = nullptr;
  HIPCHK(sdh_poll_sort(table_view(e), n, e->mt.n_lo, lo_bits, hi_bits, clo_bits, e->p_keys.p, e->p_perm.p,
                       e->p_temp.p, e->p_temp.n, e->po_q.p, e->po_key.p, e->po_ts.p, e->po_seq.p, e->po_tb.p,
                       e->po_len.p, e->po_off.p, &perm, total_words, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return perm;
}

void d2h_sync(sdh_engine* e, void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
}

void launch(sdh_engine* e, int stream, const StreamBatch& B, const int64_t t01[2],
            const std::vector<int>& qs, bool allow_chunks, bool* unordered) {
  const int64_t n = B.n;
  // chunk planning: enough waves to fill 256 CUs, chunks >> the warm-up window
  double ev_per_ms = 1.0;
  if (n > 1) ev_per_ms = (double)n / (double)std::max<int64_t>(1, t01[1] - t01[0]);
  const int64_t min_chunk = e->cfg.chunk_events > 0 ? e->cfg.chunk_events : 4096;
  const double target_waves = 16384.0;
  // every wave replays (warm-up) + emits about the same number of events, so the launch has no
  // serial tail: wave length T >= 2x the largest warm-up and ~ total work / target_waves
  double max_warm = 0;
  for (int li : qs) {
    const ChainQuery& c = e->lq[li].cq;
    if (c.chunkable) max_warm = std::max(max_warm, (double)c.within * ev_per_ms + 64.0);
  }
  const double T = std::max({2.0 * max_warm, (double)n * qs.size() / target_waves, 2.0 * min_chunk});
  e->work.clear();
  int64_t seg = 0;
  // queries grouped by state count (one kernel instantiation per group)
  std::vector<int> order(qs);
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return e->lq[a].cq.n_states < e->lq[b].cq.n_states; });
  for (int li : order) {
    const ChainQuery& c = e->lq[li].cq;
    int64_t C = 1;
    if (allow_chunks && c.chunkable) {
      const double warm = (double)c.within * ev_per_ms + 64.0;
      const double emit_len = std::max((double)min_chunk, T - warm);
      C = std::max<int64_t>(1, (int64_t)std::ceil((double)n / emit_len));
    }
    for (int64_t ch = 0; ch < C; ++ch) {
      WorkItem w{};
      w.q = li;
      w.chunk = (int)ch;
      w.n_chunks = (int)C;
      w.inb = e->cur[li];
      w.c0 = n * ch / C;
      w.c1 = n * (ch + 1) / C;
      w.seg_off = seg;
      w.seg_cap = (w.c1 - w.c0) + e->pcap + 1;
      seg += w.seg_cap;
      e->work.push_back(w);
    }
  }
  const int n_items = (int)e->work.size();
  e->d_work.ensure(n_items);
  e->d_seg_count.ensure(n_items);
  e->d_match.ensure((size_t)seg * e->rec_words);
  e->d_err.ensure(4);
  HIPCHK(hipMemcpyAsync(e->d_work.p, e->work.data(), n_items * sizeof(WorkItem), hipMemcpyHostToDevice,
                        e->stream));
  HIPCHK(hipMemsetAsync(e->d_err.p, 0, 16, e->stream));
  ChainLaunch L{};
  L.queries = e->d_q.p;
  L.work = e->d_work.p;
  L.n_work = n_items;
  L.pcap = e->pcap;
  L.b = B;
  for (int b = 0; b < 2; ++b) {
    L.hdr[b] = e->d_hdr[b].p;
    L.part[b] = e->d_part[b].p;
  }
  L.match = e->d_match.p;
  L.rec_words = e->rec_words;
  L.seg_count = e->d_seg_count.p;
  L.err = e->d_err.p;
  const size_t lds = 0;
  HIPCHK(hipEventRecord(e->ev0, e->stream));
  for (int i0 = 0; i0 < n_items;) {
    const int S = e->lq[e->work[i0].q].cq.n_states;
    int i1 = i0;
    while (i1 < n_items && e->lq[e->work[i1].q].cq.n_states == S) ++i1;
    ChainLaunch Ls = L;
    Ls.work = e->d_work.p + i0;
    Ls.seg_count = e->d_seg_count.p + i0;
    Ls.n_work = i1 - i0;
    HIPCHK(sdh_launch_chain(S, e->K, &Ls, (Ls.n_work + 3) / 4, lds, e->stream));
    i0 = i1;
  }
  HIPCHK(hipEventRecord(e->ev1, e->stream));
  int32_t errs[4];
  e->seg_count.resize(n_items);
  HIPCHK(hipMemcpyAsync(errs, e->d_err.p, 16, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(e->seg_count.data(), e->d_seg_count.p, n_items * 8, hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e->ev0, e->ev1));
  e->stats.last_kernel_ms = ms;
  if (errs[0]) throw Error(SDH_E_CAPACITY, "partial-match table overflow: raise partials_per_inst");
  if (errs[2]) throw Error(SDH_E_CAPACITY, "match segment overflow");
  *unordered = errs[1] != 0;
  // algorithmic bytes of this launch: every item streams its [w0, c1) events once
  // (approximated by c1-c0 plus warm-up), reads and writes its partial table, writes its matches
  int64_t ev_bytes = 8;
  for (int a = 0; a < B.n_attr; ++a) ev_bytes += B.width[a];
  double bytes = 0;
  int64_t total_matches = 0;
  for (int i = 0; i < n_items; ++i) {
    const WorkItem& w = e->work[i];
    const ChainQuery& c = e->lq[w.q].cq;
    double warm = w.chunk > 0 ? std::min<double>((double)w.c0, (double)c.within * ev_per_ms) : 0.0;
    bytes += ((double)(w.c1 - w.c0) + warm) * ev_bytes;
    total_matches += e->seg_count[i];
  }
  bytes += (double)qs.size() * 2.0 * NF * e->pcap * 8;  // partial tables in + out
  bytes += (double)total_matches * e->rec_words * 8;
  e->stats.last_kernel_bytes = bytes;
  e->device_matches = total_matches;
}

// ------------------------------------------------------------------------------------------
// K_ratchet host side
// ------------------------------------------------------------------------------------------
int ratchet_sim(const sdh::RatchetGroup& g);

void ratchet_build(sdh_engine* e, std::vector<std::pair<RatchetPlan, int>>& plans) {
  // lanes: normal mode in receiver-rank order (a wave's lanes are then consecutive ranks, which the
  // direct placement needs: place_cells); SDH_FLAG_DEVICE_MATCHES mode by `within`, so that similar
  // warm-up windows share a wave (SDH_RATCHET_LANES=rank|within overrides)
  const char* lo = sdh::knob("SDH_RATCHET_LANES");
  const bool by_rank = lo ? strcmp(lo, "rank") == 0 : !(e->cfg.flags & SDH_FLAG_DEVICE_MATCHES);
  const size_t ns = e->prog.stream_types.size();
  auto rank = [&](const std::pair<RatchetPlan, int>& p) { return e->out_rank[(size_t)p.second * ns + p.first.stream]; };
  std::stable_sort(plans.begin(), plans.end(), [&](const auto& a, const auto& b) {
    const auto sa = a.first.sig(), sb = b.first.sig();
    if (sa != sb) return sa < sb;
    if (by_rank) return rank(a) < rank(b);
    return a.first.within < b.first.within;
  });
  for (size_t i = 0; i < plans.size();) {
    size_t j = i;
    const auto sg = plans[i].first.sig();
    while (j < plans.size() && j - i < 64 && plans[j].first.sig() == sg) ++j;
    RatchetGroup g{};
    const RatchetPlan& P = plans[i].first;
    g.n_lanes = (int)(j - i);
    g.stream = P.stream;
    g.key_attr = P.key_attr;
    g.key_conv = P.key_conv;
    g.key_kind = P.key_kind;
    g.xmask = P.xmask;
    g.n_f0 = (int)P.f0.size();
    for (int a = 0; a < g.n_f0; ++a) g.f0[a] = P.f0[a];
    g.n_g = (int)P.g.size();
    for (int a = 0; a < g.n_g; ++a) g.g[a] = P.g[a];
    g.sim = g.n_g ? 0 : ratchet_sim(g);
    g.wmax = -1;
    for (int l = 0; l < 64; ++l) {
      const size_t k = i + std::min<size_t>(l, j - i - 1);  // idle lanes mirror the last pattern
      const RatchetPlan& Q = plans[k].first;
      g.qid[l] = plans[k].second;
      g.within[l] = Q.within < 0 ? INT64_MAX : Q.within;
      if (l < g.n_lanes) g.wmax = std::max(g.wmax, Q.within);
      for (int a = 0; a < g.n_f0; ++a) g.f0c[a][l] = Q.f0c[a];
      for (int a = 0; a < g.n_g; ++a) g.gc[a][l] = Q.gc[a];
    }
    e->rg.push_back(g);
    i = j;
  }
  // per-tile x summaries: one row per distinct (stream, key column, conversion, key kind)
  e->r_sum_specs.clear();
  for (auto& g : e->rg) {
    const std::array<int, 4> spec{g.stream, g.key_attr, g.key_conv, g.key_kind};
    int slot = -1;
    for (size_t k = 0; k < e->r_sum_specs.size(); ++k)
      if (e->r_sum_specs[k] == spec) slot = (int)k;
    if (slot < 0) {
      slot = (int)e->r_sum_specs.size();
      e->r_sum_specs.push_back(spec);
    }
    g.sum_slot = slot;
  }
  const size_t ng = e->rg.size();
  e->rcur.assign(ng, 0);
  e->r_full_expiry.assign(e->prog.stream_types.size(), 0);
  if (!ng) return;
  e->d_rg.ensure(ng);
  HIPCHK(hipMemcpy(e->d_rg.p, e->rg.data(), ng * sizeof(RatchetGroup), hipMemcpyHostToDevice));
  for (int b = 0; b < 2; ++b) {
    e->d_rst[b].ensure(ng);
    HIPCHK(hipMemset(e->d_rst[b].p, 0, ng * sizeof(RatchetState)));
    e->d_rts[b].ensure(ng * e->rsmax * WAVE);
    e->d_rsq[b].ensure(ng * e->rsmax * WAVE);
    e->d_rky[b].ensure(ng * e->rsmax * WAVE);
  }
  e->d_blk_next.ensure(4);
}

// persisted deques with room for `want` entries per lane: [g][rsmax][64] re-strided (both buffers)
void ratchet_grow_rsmax(sdh_engine* e, int64_t want) {
  if (want <= e->rsmax) return;
  int64_t cap = e->rsmax;
  while (cap < want) cap *= 2;
  const size_t ng = e->rg.size(), ob = (size_t)e->rsmax * WAVE * 8, nb = (size_t)cap * WAVE * 8;
  for (int b = 0; b < 2; ++b)
    for (DevBuf<int64_t>* buf : {&e->d_rts[b], &e->d_rsq[b], &e->d_rky[b]}) {
      DevBuf<int64_t> nw;
      nw.ensure(ng * cap * WAVE);
      HIPCHK(hipMemcpy2DAsync(nw.p, nb, buf->p, ob, ob, ng, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      std::swap(buf->p, nw.p);
      std::swap(buf->n, nw.n);
    }
  e->rsmax = cap;
}

int64_t ratchet_count_matches(sdh_engine* e) {
  int64_t n = 0;
  for (int i = 0; i < e->r_blocks_used; ++i) n += e->r_blk_count[i];
  return n;
}

// one NFA step of every ratchet group fed by `stream` over batch B (exact re-runs on overflow /
// out-of-order timestamps: the groups' input deques are double-buffered and untouched until the
// launch succeeds)
// f0 atoms a K_ratchet launch variant must handle: the one-atom variant assumes a constant
// interval, so a group with a two-column atom (`cur.a OP cur.b`) takes the general variant
int ratchet_nf(const sdh::RatchetGroup& g) {
  for (int a = 0; a < g.n_f0; ++a)
    if (g.f0[a].cur2) return sdh::RMAXF0;
  return g.n_f0;
}

// the SIM form (nfa_ratchet.hip): float keys from a float column, one start atom over that same
// column compared in the float / double domain against a constant, without negation
int ratchet_sim(const sdh::RatchetGroup& g) {
  if (sdh::knob("SDH_RATCHET_NO_SIM")) return 0;
  if (g.key_kind != sdh::KK_F32 || g.key_conv == sdh::CV_F32_INT || g.key_conv == sdh::CV_F32_LONG || g.n_f0 != 1)
    return 0;
  const sdh::RatchetAtom& A = g.f0[0];
  return (A.attr == g.key_attr && !A.cur2 && A.f64 && (A.conv == sdh::CV_F32_FLOAT || A.conv == sdh::CV_F64_FLOAT) &&
          !(A.mask & sdh::CM_NOT)) ? 1 : 0;
}

void launch_ratchet(sdh_engine* e, int stream, const StreamBatch& B, const int64_t t01[2]) {
  e->r_placing = false;
  e->r_blocks_used = 0;
  e->r_matches = 0;
  e->r_kernel_ms = 0;
  e->r_kernel_bytes = 0;
  e->r_rec_bytes = 0;
  e->r_rec4 = 0;
  std::vector<int> gs;
  for (int g = 0; g < (int)e->rg.size(); ++g)
    if (e->rg[g].stream == stream) gs.push_back(g);
  if (gs.empty()) return;
  const int64_t n = B.n;
  int64_t lanes = 0;
  for (int g : gs) lanes += e->rg[g].n_lanes;
  const bool devrec = (e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) != 0;
  if (e->r_blocks == 0) {
    // a first guess (at most 8 GiB of blocks): a push that needs more re-runs once with the count of
    // blocks its waves asked for
    int64_t want = e->cfg.match_capacity > 0 ? e->cfg.match_capacity : std::max<int64_t>(1 << 20, n * lanes * 3 / 4);
    if (e->cfg.match_capacity <= 0) want = std::min<int64_t>(want, (int64_t)1 << 30);
    e->r_blocks = (want + e->r_blk_recs - 1) / e->r_blk_recs;
  }
  e->d_rtotal.ensure(3);  // [0] device-record entries, [1] the placement total, [2] device-record bytes
  bool no_place = false, no_rec4 = false;
  for (int attempt = 0; attempt < 40; ++attempt) {
    // out-of-order timestamps seen on this stream, timestamps so extreme that `ts0 + within`
    // could wrap, or a batch spanning 2^31 - 2 ms or more (the lazy forms' 32-bit deadline domain,
    // nfa_ratchet.hip rel_deadline): exact per-entry expiry scan, no chunking
    const int64_t lim = (int64_t)1 << 61;
    const bool full = e->r_full_expiry[stream] != 0 || t01[0] < -lim || t01[0] > lim || t01[1] < -lim ||
                      t01[1] > lim || (B.prev_ts != INT64_MIN && (B.prev_ts < -lim || B.prev_ts > lim)) ||
                      t01[1] - t01[0] > (int64_t)INT32_MAX - 2;
    // ---- chunk planning: chunk c > 0 rebuilds its starting deques by a reverse scan of the
    // `within` window (a few instructions per 64 events), so chunks can be short. Each launch
    // (one key kind x orientation) gets one resident wave per slot of the chip -- CUs x the
    // kernel's occupancy -- of at least min_chunk emitted events each ----
    // (C2 expansion, 64K-event pushes, tools/sweep_minchunk.sh: 2,048 events per chunk at least
    // 3.66 ms per push / 3.56 compact, 1,024 3.42 / 3.43, 512 3.43 / 3.48, 256 3.68 / 3.68)
    const int64_t def_chunk = sdh::knob("SDH_RATCHET_MIN_CHUNK") ? atoll(sdh::knob("SDH_RATCHET_MIN_CHUNK")) : 1024;
    const int64_t min_chunk = e->cfg.chunk_events > 0 ? e->cfg.chunk_events : def_chunk;
    e->ritems.clear();
    std::vector<int> order(gs);
    // launches: one per (key kind, orientation, SIM form); SIM also needs the key column null-free
    // in this batch
    auto lsim = [&](int g) { return e->rg[g].sim && !B.nul[e->rg[g].key_attr] ? 1 : 0; };
    auto lgate = [&](int g) { return e->rg[g].n_g > 0 ? 1 : 0; };  // K_gate groups (nfa_gate.hip)
    auto lkey = [&](int g) { return std::make_tuple(lgate(g), e->rg[g].key_kind, e->rg[g].xmask, lsim(g)); };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return lkey(a) < lkey(b); });
    for (size_t i0 = 0; i0 < order.size();) {
      size_t i1 = i0;
      int nf = 0;
      while (i1 < order.size() && lkey(order[i1]) == lkey(order[i0])) nf = std::max(nf, ratchet_nf(e->rg[order[i1++]]));
      // items per launch: 8 rounds of the chip's resident slots (CUs x occupancy). Short chunks
      // balance the groups' uneven match density, and a chunk's reverse-scan warm-up is cheap (tile
      // summaries). C2 at 10K patterns, tools/sweep_ratchet.sh (SDH_RATCHET_WAVES): 8,192 items
      // 117.8 ms/step, 16,384 110.9, 32,768 103.3, 65,536 100.2, 131,072 100.8, 524,288 104.4
      double slots = e->r_waves;
      if (slots <= 0) {
        const int occ = lgate(order[i0]) ? sdh_gate_occupancy(nf, nf)
                                         : sdh_ratchet_occupancy(e->rg[order[i0]].key_kind, full, nf, e->rML, lsim(order[i0]));
        slots = 8.0 * (double)e->n_cu * std::max(1, occ);
      }
      // chunks per chunkable group: as many as fit the item target (floor, not ceil: a partial
      // extra round of items runs as a nearly idle tail -- C2 at 10K once had 8,321 items for 8,192
      // slots, 128.7 ms/step, against 117.7 at 8,164), at least min_chunk events each. Groups
      // without `within` cannot chunk (no reverse-scan window) and hold one item each.
      int64_t n_chunkable = 0;
      for (size_t i = i0; i < i1; ++i) n_chunkable += (!full && e->rg[order[i]].wmax >= 0) ? 1 : 0;
      const int64_t free_slots = std::max<int64_t>(1, (int64_t)slots - ((int64_t)(i1 - i0) - n_chunkable));
      const int64_t c_fit = n_chunkable > 0 ? std::max<int64_t>(1, free_slots / n_chunkable) : 1;
      const int64_t c_min = std::max<int64_t>(1, n / std::max<int64_t>(1, min_chunk));
      for (size_t i = i0; i < i1; ++i) {
        const int g = order[i];
        const RatchetGroup& G = e->rg[g];
        int64_t C = 1;
        if (!full && G.wmax >= 0) {
          C = std::min(c_fit, c_min);
          // a chunk's warm-up walks its `within` window back from its first event: tiles whose best
          // key is dominated by the later ones are skipped on their summary, but flat or rising key
          // runs are walked event by event. Chunks x window events <= max(16 x the batch, 2^24)
          // bounds that worst case (a 67M-event window spanning the batch: 16 chunks) and binds
          // nowhere near C2's windows (1-60 s, up to 60K events, in 8M- or 64K-event pushes)
          const double span = (double)std::max<int64_t>(1, t01[1] - t01[0]);
          const double win_ev = std::min((double)n, (double)G.wmax * (double)n / span);
          const double budget = std::max(16.0 * (double)n, 16777216.0);
          C = std::min<int64_t>(C, std::max<int64_t>(1, (int64_t)(budget / std::max(1.0, win_ev))));
        }
        for (int64_t ch = 0; ch < C; ++ch) {
          RatchetItem it{};
          it.g = g;
          it.chunk = (int)ch;
          it.n_chunks = (int)C;
          it.inb = e->rcur[g];
          it.c0 = n * ch / C;
          it.c1 = n * (ch + 1) / C;
          e->ritems.push_back(it);
        }
      }
      i0 = i1;
    }
    const int n_items = (int)e->ritems.size();
    e->d_ritems.ensure(n_items);
    HIPCHK(hipMemcpyAsync(e->d_ritems.p, e->ritems.data(), n_items * sizeof(RatchetItem),
                          hipMemcpyHostToDevice, e->stream));
    // 8-B records address e2 by a 26-bit batch offset; larger batches use 16-B records. A placing
    // launch writes no records: COUNT, scan, WRITE (compact rows)
    const bool placing = !no_place && ratchet_placeable(e, stream, B.seq_base, n, full);
    const int wide = n > ((int64_t)1 << 26) ? 1 : 0;
    if (n > ((int64_t)1 << 32)) throw Error(SDH_E_INVALID, "batch larger than 2^32 events");
    e->d_rmatch.ensure((size_t)(e->r_blocks + 1) * e->r_blk_recs * (wide ? 2 : 1));  // (+ the spare block)
    e->d_rspillA.ensure((size_t)n_items * e->rSC * WAVE);
    e->d_rlts.ensure((size_t)n_items * e->rML * WAVE);
    bool any64 = false;
    for (int g : gs) any64 |= e->rg[g].key_kind == KK_F64 || e->rg[g].key_kind == KK_I64;
    if (any64) e->d_rspillB.ensure((size_t)n_items * e->rSC * WAVE);
    e->d_blk_count.ensure((size_t)e->r_blocks);
    e->d_blk_group.ensure((size_t)e->r_blocks);
    e->d_blk_side.ensure((size_t)e->r_blocks);
    e->d_err.ensure(5);
    HIPCHK(hipMemsetAsync(e->d_err.p, 0, 20, e->stream));
    HIPCHK(hipMemsetAsync(e->d_blk_next.p, 0, 4, e->stream));
    HIPCHK(hipMemsetAsync(e->d_rtotal.p, 0, 24, e->stream));
    // per-tile x summaries for the warm-up scans (rows of this stream's key specs)
    const int64_t n_tiles = (n + 63) / 64;
    const size_t n_rows = e->r_sum_specs.size();
    e->d_tsmax.ensure(n_rows * n_tiles);
    e->d_tsmin.ensure(n_rows * n_tiles);
    e->d_tshas.ensure(n_rows * n_tiles);
    if (!full)
      for (size_t r = 0; r < n_rows; ++r) {
        const auto& sp = e->r_sum_specs[r];
        if (sp[0] != stream) continue;
        HIPCHK(sdh_launch_ratchet_summary(sp[3], &B, sp[1], sp[2], n_tiles, e->d_tsmax.p + r * n_tiles,
                                          e->d_tsmin.p + r * n_tiles, e->d_tshas.p + r * n_tiles, e->stream));
      }
    RatchetLaunch L{};
    L.groups = e->d_rg.p;
    L.full_expiry = full;
    L.tsum_max = e->d_tsmax.p;
    L.tsum_min = e->d_tsmin.p;
    L.tsum_has = e->d_tshas.p;
    L.n_tiles = n_tiles;
    L.b = B;
    L.rsmax = e->rsmax;
    for (int b = 0; b < 2; ++b) {
      L.st[b] = e->d_rst[b].p;
      L.ent_ts[b] = e->d_rts[b].p;
      L.ent_seq[b] = e->d_rsq[b].p;
      L.ent_key[b] = e->d_rky[b].p;
    }
    L.spillA = e->d_rspillA.p;
    L.spillB = e->d_rspillB.p;
    L.match = e->d_rmatch.p;
    L.blk_count = e->d_blk_count.p;
    L.blk_side = e->d_blk_side.p;
    // device records take the 4-B rec4 entries where they can
    L.rec4 = (devrec && !wide && !full && !no_rec4) ? 1 : 0;
    L.blk_group = e->d_blk_group.p;
    L.wide = wide;
    L.blk_next = e->d_blk_next.p;
    L.n_blocks = (int32_t)std::min<int64_t>(e->r_blocks, INT32_MAX);
    L.blk_recs = e->r_blk_recs;
    L.dev_records = devrec ? 1 : 0;
    L.rec_total = e->d_rtotal.p;
    L.err = e->d_err.p;
    const int nc = e->place_cells[(size_t)stream];
    const int64_t cells = n * nc + 1;  // (+1: the scan's total)
    if (placing) {
      e->p_cnt.ensure((size_t)cells);
      HIPCHK(hipMemsetAsync(e->p_cnt.p + cells - 1, 0, 4, e->stream));
      L.pcnt = e->p_cnt.p;
      L.n_cells = nc;
    }
    e->r_placing = false;
    int any_rec4 = 0;
    // one launch per (key kind, orientation, SIM form)
    auto run = [&](const RatchetLaunch& L0) {
      for (int i0 = 0; i0 < n_items;) {
        const int g0 = e->ritems[i0].g;
        const int kk = e->rg[g0].key_kind, xm = e->rg[g0].xmask, sim = lsim(g0), gate = lgate(g0);
        int i1 = i0;
        while (i1 < n_items && lkey(e->ritems[i1].g) == lkey(g0)) ++i1;
        RatchetLaunch Ls = L0;
        Ls.items = e->d_ritems.p + i0;
        Ls.n_items = i1 - i0;
        int nf = 0;
        for (int i = i0; i < i1; ++i) nf = std::max(nf, ratchet_nf(e->rg[e->ritems[i].g]));
        // spill regions are indexed by the item's position in its launch
        Ls.spillA = e->d_rspillA.p + (size_t)i0 * e->rSC * WAVE;
        Ls.lds_ts = e->d_rlts.p + (size_t)i0 * e->rML * WAVE;
        Ls.spillB = any64 ? e->d_rspillB.p + (size_t)i0 * e->rSC * WAVE : nullptr;
        Ls.rec4 = L0.rec4 && sim && !gate ? 1 : 0;  // (rec4 blocks come from the SIM form only)
        any_rec4 |= Ls.rec4;
        if (gate) {
          int ng = 0;
          for (int i = i0; i < i1; ++i) ng = std::max(ng, e->rg[e->ritems[i].g].n_g);
          HIPCHK(sdh_launch_gate(kk, xm, full, nf, ng, e->rSC, &Ls, e->stream));
        } else {
          HIPCHK(sdh_launch_ratchet(kk, xm, full, nf, full ? 0 : sim, e->rML, e->rSC, &Ls, e->stream));
        }
        i0 = i1;
      }
    };
    HIPCHK(hipEventRecord(e->ev0, e->stream));
    run(L);
    HIPCHK(hipEventRecord(e->ev1, e->stream));
    int32_t errs[5], used = 0;
    HIPCHK(hipMemcpyAsync(errs, e->d_err.p, 20, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&used, e->d_blk_next.p, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e->ev0, e->ev1));
    if (sdh::knob("SDH_TRACE"))
      fprintf(stderr, "[sdh] ratchet stream %d n %lld attempt %d full %d rec4 %d items %d blocks %d/%lld errs %d %d %d %d %d: %.2f ms\n",
              stream, (long long)n, attempt, (int)full, L.rec4, n_items, used, (long long)e->r_blocks, errs[0], errs[1],
              errs[2], errs[3], errs[4], ms);
    if (errs[3]) throw Error(SDH_E_CAPACITY, "a pending partial is more than 2^31 events old");
    if (errs[1] && !full) {  // timestamps out of order: exact re-run with the full expiry scan
      e->r_full_expiry[stream] = 1;
      continue;
    }
    if (errs[0]) {
      // exact re-run with a larger spill ring (and persisted deques to hold it): the reference's
      // pending list is unbounded (StreamPreStateProcessor.java:298)
      if (e->rSC >= (1 << 24))
        throw Error(SDH_E_CAPACITY, fmt("more than %d pending partials in one pattern", e->rML + e->rSC));
      e->rSC *= 2;
      ratchet_grow_rsmax(e, e->rML + e->rSC);
      continue;
    }
    if (errs[2]) {
      // out of blocks: blk_next ends at the number of blocks the launch's waves asked for (a wave past
      // the last block writes into the spare one and keeps counting), so one re-run with that many fits
      const int64_t need = std::max<int64_t>(2 * e->r_blocks, (int64_t)used + used / 64 + 64);
      const int64_t blk_bytes = (int64_t)e->r_blk_recs * 8 * (wide ? 2 : 1);
      size_t fr = 0, tot = 0;
      HIPCHK(hipMemGetInfo(&fr, &tot));
      const double have = (double)fr + (double)e->d_rmatch.n * 8.0 - (double)(1 << 30);
      int64_t nb = std::max<int64_t>((int64_t)used + used / 64 + 64, e->r_blocks + 1);
      if ((double)(need + 1) * blk_bytes <= have) nb = std::max(nb, need);
      if ((double)(nb + 1) * blk_bytes > have || nb >= INT32_MAX)
        throw Error(SDH_E_CAPACITY, fmt("the push's match records need %.1f GB of HBM (%.1f GB free): push fewer events "
                                        "per call", (double)(nb + 1) * blk_bytes / 1e9, have / 1e9));
      e->r_blocks = nb;
      continue;
    }
    if (errs[4] && L.rec4) {  // a rec4 entry's e1 distance reached 2^26: exact re-run with 8-B records
      no_rec4 = true;  // (this push only: the next one tries rec4 again)
      ++e->r_rec4_reruns;
      continue;
    }
    int64_t placed_rows = 0;
    if (placing) {
      // the (event, cell) counts -> each cell's first row; then the same items again, writing
      e->p_ptemp.ensure(sdh_place_temp_bytes(cells));
      HIPCHK(sdh_place_total(e->p_cnt.p, cells, e->d_rtotal.p + 1, e->stream));
      HIPCHK(sdh_place_scan(e->p_cnt.p, cells, e->p_ptemp.p, e->p_ptemp.n, e->stream));
      unsigned long long tot = 0;
      HIPCHK(hipMemcpyAsync(&tot, e->d_rtotal.p + 1, 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      placed_rows = (int64_t)tot;
      const int64_t n0 = e->mt.n;
      if (tot >= (unsigned long long)INT32_MAX || n0 + placed_rows >= INT32_MAX) {  // (2^31 rows: table records)
        no_place = true;
        continue;
      }
      e->pc_rows.grow_keep((size_t)((n0 + placed_rows) * e->cw), (size_t)(n0 * e->cw), e->stream);
      RatchetLaunch W = L;
      W.pcnt = nullptr;
      W.pbase = e->p_cnt.p;
      W.crow = e->pc_rows.p;
      W.cw = e->cw;
      W.row0 = n0;
      e->r_place_row0 = n0;
      W.seq_ref = e->seq_ref;
      float ms2 = 0;
      HIPCHK(hipEventRecord(e->ev0, e->stream));
      run(W);
      HIPCHK(hipEventRecord(e->ev1, e->stream));
      HIPCHK(hipEventSynchronize(e->ev1));
      HIPCHK(hipEventElapsedTime(&ms2, e->ev0, e->ev1));
      ms += ms2;
    }
    for (int g : gs) e->rcur[g] ^= 1;
    e->r_placing = placing;
    e->r_blk_taken = used;
    e->r_seq_base = B.seq_base;
    if (placing) {
      e->r_blocks_used = 0;
      e->r_matches = placed_rows;
    } else if (devrec) {  // left on the device for sdh_engine_poll_records: the blocks 0 .. used-1
      unsigned long long tot[3] = {0, 0, 0};
      HIPCHK(hipMemcpy(tot, e->d_rtotal.p, 24, hipMemcpyDeviceToHost));
      e->r_blocks_used = used;
      e->r_matches = (int64_t)tot[0];
      e->r_rec_bytes = (double)tot[2];
      e->r_rec4 = any_rec4;
    } else {
      e->r_blocks_used = std::min<int>(used, (int)e->r_blocks);
      e->r_blk_count.resize(e->r_blocks_used);
      if (e->r_blocks_used)
        HIPCHK(hipMemcpy(e->r_blk_count.data(), e->d_blk_count.p, e->r_blocks_used * 4, hipMemcpyDeviceToHost));
      e->r_matches = ratchet_count_matches(e);
    }
    e->r_kernel_ms = ms;
    e->r_wide = wide;
    // algorithmic bytes: every group streams the batch's operand columns once
    // (ts + x-atom column + f0 columns; the warm-up re-reads are overhead, not counted), writes
    // 32 B per match (SURVEY §8(d)'s unit; the device record is 8 B, expanded at poll) and reads +
    // writes its persisted deques (24 B per pending partial)
    double bytes = 0;
    for (int g : gs) {
      const RatchetGroup& G = e->rg[g];
      int64_t ev_bytes = 8 + B.width[G.key_attr];
      for (int a = 0; a < G.n_f0; ++a) {
        if (G.f0[a].attr != G.key_attr) ev_bytes += B.width[G.f0[a].attr];
        if (G.f0[a].cur2 && G.f0[a].attr2 != G.key_attr) ev_bytes += B.width[G.f0[a].attr2];
      }
      for (int a = 0; a < G.n_g; ++a)  // (K_gate's gate columns)
        if (G.g[a].attr != G.key_attr) ev_bytes += B.width[G.g[a].attr];
      bytes += (double)n * ev_bytes;
    }
    bytes += (double)e->r_matches * 32.0;
    e->r_kernel_bytes = bytes;
    return;
  }
  throw Error(SDH_E_CAPACITY, "ratchet launch did not converge");
}

// ------------------------------------------------------------------------------------------
// K_gen host side: lowering, instance arenas, partition routing, launch, match collection
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// K_part shape selection (nfa_part.hip): partitioned `every e1 -> (e2 and|or e3)` and
// `every e1 -> e2<min:max> -> e3` patterns whose structure the compact partial tables reproduce
// exactly (the argument is in nfa_part.hip's header)
// ------------------------------------------------------------------------------------------
struct KPart {
  int kind = -1, sA = 1, sB = 2, cmax = 0, n_e1 = 0, n_first = 0, n_last = 0;
};

// every slot reference of state i's filters: (slot, chain index) pairs; false if an instruction
// names a slot in another way than OP_ATTR / OP_STREAM_IS_NULL
void filter_refs(const kg::LState& st, std::vector<std::pair<int64_t, int64_t>>& refs) {
  for (const auto& f : st.filters)
    for (const auto& in : f)
      if (in.op == kg::OP_ATTR || in.op == kg::OP_STREAM_IS_NULL) refs.push_back({in.a, in.b});
}

KPart kpart_shape(const kg::LProgram& P, int qi, const kg::GQuery& g) {
  KPart k;
  const kg::LQuery& q = P.q[qi];
  if (q.partition < 0 || q.type != kg::Q_PATTERN || q.st.size() != 3) return k;
  for (const auto& x : q.st)
    if (x.waiting != -1) return k;  // absent sides run on K_gen
  // start ids exist only with `within` (StateInputStreamParser.java:126-138): then e1 alone
  if (!(q.start_ids.empty() || (q.start_ids.size() == 1 && q.start_ids[0] == 0)) || g.max_depth > kg::RSTACK) return k;
  if (q.start_ids.empty() && q.within >= 0) return k;
  const int s = q.st[0].stream;
  for (const auto& x : q.st)
    if (x.stream != s || x.within_every != -1 || x.callback != -1) return k;
  if (q.recvs.size() != 1 || q.recvs[0].stream != s || q.recvs[0].procs.size() != 3 || q.recvs[0].procs[0] != 0)
    return k;
  const kg::LState& e1 = q.st[0];
  if (e1.kind != kg::K_STREAM || !e1.is_start || e1.next_every != 0 || e1.has_selector) return k;
  std::vector<std::pair<int64_t, int64_t>> r;
  const auto& procs = q.recvs[0].procs;
  if (q.st[1].kind == kg::K_LOGICAL) {
    const kg::LState &a = q.st[1], &b = q.st[2];
    if (b.kind != kg::K_LOGICAL || a.partner != 2 || b.partner != 1 || a.ltype != b.ltype) return k;
    for (const auto* x : {&a, &b})
      if (x->is_start || x->next_pre != -1 || x->next_every != -1 || !x->has_selector) return k;
    if (e1.next_pre != 1 && e1.next_pre != 2) return k;
    if (!((procs[1] == 1 && procs[2] == 2) || (procs[1] == 2 && procs[2] == 1))) return k;
    for (int i = 1; i <= 2; ++i) {  // the sides' filters read only their own slot (event-only)
      r.clear();
      filter_refs(q.st[i], r);
      for (const auto& x : r)
        if (x.first != i) return k;
    }
    k.sA = procs[1];  // registration order: the side processed second
    k.sB = procs[2];
    k.kind = a.ltype == kg::L_AND ? PK_AND : PK_OR;
    return k;
  }
  const kg::LState &c = q.st[1], &e3 = q.st[2];
  if (c.kind != kg::K_COUNT || c.min < 1 || c.max > PK_CMAX || c.min > c.max) return k;
  if (c.next_pre != 2 || c.next_every != -1 || c.has_selector || e1.next_pre != 1) return k;
  if (e3.kind != kg::K_STREAM || e3.next_pre != -1 || e3.next_every != -1 || !e3.has_selector) return k;
  if (procs[1] != 1 || procs[2] != 2) return k;
  r.clear();
  filter_refs(c, r);  // the count filter reads only the event it is appending (CURRENT)
  for (const auto& x : r)
    if (x.first != 1 || x.second != -1) return k;
  r.clear();
  filter_refs(e3, r);  // e3 reads e1, e2[0], e2[last] (= CURRENT of another state) and itself
  const int ncap = g.n_cap[s];
  for (const auto& x : r) {
    if (x.first == 1) {
      if (x.second == 0) k.n_first = ncap;
      else if (x.second == -1) k.n_last = ncap;
      else return k;
    } else if (x.first == 0) {
      k.n_e1 = ncap;
    }
  }
  r.clear();
  filter_refs(e1, r);
  k.cmax = c.max;
  k.kind = PK_COUNT;
  return k;
}

// Shape-compiled kernels (spec.h): SDH_SPEC=0 none, 1 every shape, "require" every shape and a
// failed compile is an error; default: shapes that fill at least two waves (a compile costs about
// a second once per process and shape, the interpreted kernel is exact too)
int spec_mode() {
  const char* v = sdh::knob("SDH_SPEC");
  if (!v || !*v) return 1;
  if (!strcmp(v, "0")) return 0;
  if (!strcmp(v, "require")) return 3;
  return 2;
}

void spec_build(sdh_engine* e) {
  const int mode = spec_mode();
  if (mode == 0) return;
  std::map<int, int> groups;  // K_seq template -> groups
  for (size_t g = 0; g < e->group_seq.size(); ++g)
    if (e->group_seq[g] > 0) ++groups[e->group_tmpl[g]];
  for (const auto& [t, ng] : groups) {
    if (mode == 1 && ng < 2) continue;
    std::string err;
    // ring-mode output reserves the ring in chunks (dev_common.h SDH_RING_CHUNK), so its flushes are
    // cheap and a smaller LDS buffer buys resident waves (C4 ring: 1024 words 25.9 ms/step, 768 22.9,
    // 512 23.7); normal-mode flushes take two atomics each and keep the larger buffer
    const int seq_w = (e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) ? 768 : 0;
    hipFunction_t f = sdh::spec::get_kernel(sdh::spec::seq_source(e->gq[t], seq_w), "sdh_seq_spec", &err);
    if (!f && mode == 3) throw Error(SDH_E_DEVICE, "shape-compiled K_seq kernel: " + err);
    if (f) e->seq_spec[t] = f;
  }
  int64_t n = (int64_t)e->seq_spec.size();
  for (auto& up : e->psets) {
    auto& ps = *up;
    std::map<int, int> pg;  // template -> groups
    for (int g = 0; g < ps.n_groups; ++g) ++pg[e->group_tmpl[ps.group_base + g]];
    for (const auto& [t, ng] : pg) {
      if (mode == 1 && ng < 2) continue;
      // register-resident entries per lane: the first few partials of a (query, key) instance
      // stay in VGPRs across the key's events (C3 instances hold a handful at a time)
      // (C3 at 1000 x 10K keys, or/and entries: 8 26.0 ms/step, 6 25.4, 5 25.1, 4 24.6, 3 24.4, 2 32.8)
      int regs = ps.kind == PK_COUNT ? 3 : 3;
      if (const char* v = sdh::knob(ps.kind == PK_COUNT ? "SDH_KPART_REGS_COUNT" : "SDH_KPART_REGS")) regs = std::max(0, atoi(v));
      sdh::spec::PartLayout lay{ps.kind, ps.sA, ps.sB, ps.cmax, ps.n_e1, ps.n_first, ps.n_last, ps.ew, regs};
      // (C3 ring: 1536 words 20.7 ms/step, 1024 17.5, 768 18.0, 2048 21.8)
      if (e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) lay.out_w = 1024;
      std::string err;
      hipFunction_t f = sdh::spec::get_kernel(sdh::spec::part_source(e->gq[t], lay), "sdh_part_spec", &err);
      if (!f && mode == 3) throw Error(SDH_E_DEVICE, "shape-compiled K_part kernel: " + err);
      if (f) ps.spec[t] = f, ++n;
    }
  }
  e->stats.spec_kernels = n;
}

// ------------------------------------------------------------------------------------------
// K_slab host side (nfa_slab.hip): directory growth with the key table, slab space (reclaiming a
// sub-ring's oldest half, growing), rollback of a failed push
// ------------------------------------------------------------------------------------------
void slab_heads(sdh_engine* e, sdh_engine::SlabSet& ss) {
  ss.h_head.resize(ss.nsub);
  HIPCHK(hipMemcpyAsync(ss.h_head.data(), ss.head.p, ss.nsub * 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
}

void slab_upload_rings(sdh_engine::SlabSet& ss) {
  HIPCHK(hipMemcpy(ss.d_ring.p, ss.ring.data(), ss.nsub * sizeof(uint32_t*), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ss.d_cap.p, ss.cap.data(), ss.nsub * 8, hipMemcpyHostToDevice));
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

uint32_t* ring_malloc(sdh_engine* e, sdh_engine::SlabSet& ss, int64_t words) {
  (void)e;
  uint32_t* p = ss.alloc_ring(words);
  if (!p) throw Error(SDH_E_CAPACITY, fmt("device memory exhausted allocating a %.2f GB K_slab ring", words * 4.0 / 1e9));
  return p;
}

// fresh, empty sub-rings of `cap` words each
void slab_init(sdh_engine* e, sdh_engine::SlabSet& ss, int64_t cap) {
  for (size_t r = 0; r < ss.ring.size(); ++r) ss.free_ring(ss.ring[r], r < ss.cap.size() ? ss.cap[r] : 0);
  cap = (cap + 3) & ~3ll;
  ss.ring.assign(ss.nsub, nullptr);
  ss.cap.assign(ss.nsub, cap);
  for (auto& p : ss.ring) p = ring_malloc(e, ss, cap);
  ss.d_ring.ensure(ss.nsub);
  ss.d_cap.ensure(ss.nsub);
  slab_upload_rings(ss);
  ss.head.ensure(ss.nsub);
  ss.tail.ensure(ss.nsub);
  ss.head_bak.ensure(ss.nsub);
  HIPCHK(hipMemset(ss.head.p, 0, ss.nsub * 8));
  HIPCHK(hipMemset(ss.tail.p, 0, ss.nsub * 8));
  ss.h_head.assign(ss.nsub, 0);
  ss.h_tail.assign(ss.nsub, 0);
  ss.h_push0.assign(ss.nsub, 0);
  ss.live.ensure(256);
  ss.live_bak.ensure(256);
  ss.traffic.ensure(256);
  HIPCHK(hipMemset(ss.live.p, 0, 256 * 8));
}

// directory room for `keys` keys (key-major: the old entries are a prefix; new keys' blocks empty)
void slab_grow_keys(sdh_engine* e, sdh_engine::SlabSet& ss, int64_t keys) {
  if (keys <= ss.key_cap) return;
  int64_t cap = std::max<int64_t>(64, ss.key_cap);
  while (cap < keys) cap *= 2;
  const size_t old_n = (size_t)ss.key_cap * ss.n_groups, new_n = (size_t)cap * ss.n_groups;
  DevBuf<uint64_t> nd;
  if (hipMalloc(&nd.p, new_n * 8) != hipSuccess)
    throw Error(SDH_E_CAPACITY, fmt("device memory exhausted growing the K_slab directory to %lld keys", (long long)cap));
  nd.n = new_n;
  HIPCHK(hipMemsetAsync(nd.p + old_n, 0, (new_n - old_n) * 8, e->stream));
  if (old_n) HIPCHK(hipMemcpyAsync(nd.p, ss.dir.p, old_n * 8, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::swap(ss.dir.p, nd.p);
  std::swap(ss.dir.n, nd.n);
  ss.key_cap = cap;
}

// One directory pass moving blocks (nfa_slab.hip slab_move_kernel); false if a destination ring
// ran out of room (nothing is lost: a block keeps its old place until its directory word moves)
bool slab_move_raw(sdh_engine* e, sdh_engine::SlabSet& ss, uint64_t* dir, uint32_t* const* src_ring,
                   const int64_t* src_cap, const unsigned long long* src_tail, int src_nsub,
                   const std::vector<unsigned long long>& limit, const std::vector<uint8_t>& active,
                   uint32_t* const* dst_ring, const int64_t* dst_cap, unsigned long long* dst_head,
                   const unsigned long long* dst_tail, int dst_nsub, std::vector<uint8_t>* ring_fail = nullptr) {
  DevBuf<unsigned long long> d_lim;
  DevBuf<uint8_t> d_act;
  d_lim.ensure(limit.size());
  HIPCHK(hipMemcpyAsync(d_lim.p, limit.data(), limit.size() * 8, hipMemcpyHostToDevice, e->stream));
  if (!active.empty()) {
    d_act.ensure(active.size());
    HIPCHK(hipMemcpyAsync(d_act.p, active.data(), active.size(), hipMemcpyHostToDevice, e->stream));
  }
  e->d_err.ensure(4);
  HIPCHK(hipMemsetAsync(e->d_err.p, 0, 16, e->stream));
  DevBuf<uint8_t> d_rf;
  if (ring_fail) {
    d_rf.ensure(dst_nsub);
    HIPCHK(hipMemsetAsync(d_rf.p, 0, dst_nsub, e->stream));
  }
  HIPCHK(sdh_slab_move(dir, ss.key_cap * ss.n_groups, ss.n_groups, ss.d_group_ew.p, src_ring, src_cap, src_tail,
                       src_nsub, d_lim.p, active.empty() ? nullptr : d_act.p, dst_ring, dst_cap, dst_head, dst_tail,
                       dst_nsub, e->d_err.p, ring_fail ? d_rf.p : nullptr, e->stream));
  int32_t err = 0;
  HIPCHK(hipMemcpyAsync(&err, e->d_err.p, 4, hipMemcpyDeviceToHost, e->stream));
  if (ring_fail) {
    ring_fail->assign(dst_nsub, 0);
    HIPCHK(hipMemcpyAsync(ring_fail->data(), d_rf.p, dst_nsub, hipMemcpyDeviceToHost, e->stream));
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  return err == 0;
}

// rings `which` into new buffers of new_cap[r] words holding their live blocks (a batch at a time,
// so the extra memory is a batch's worth)
void slab_grow(sdh_engine* e, sdh_engine::SlabSet& ss, const std::vector<int>& which,
               const std::vector<int64_t>& new_cap) {
  // (up to 32 rings and 8 GB of new buffers at a time: old and new buffers coexist while a batch
  // moves, and C5's rings reach GBs each -- 32 at a time took tens of GB on top of the state)
  const int BATCH = 32;
  const int64_t BATCH_WORDS = (int64_t)2 << 30;
  for (size_t b0 = 0, b1 = 0; b0 < which.size(); b0 = b1) {
    const double t_start = now_ms();
    std::vector<uint32_t*> nring(ss.ring);
    std::vector<int64_t> ncap(ss.cap);
    std::vector<uint8_t> active(ss.nsub, 0);
    int64_t words = 0;
    for (b1 = b0; b1 < which.size() && b1 < b0 + BATCH && (b1 == b0 || words + new_cap[b1] <= BATCH_WORDS); ++b1) {
      const int r = which[b1];
      ncap[r] = (new_cap[b1] + 3) & ~3ll;
      nring[r] = ring_malloc(e, ss, ncap[r]);
      active[r] = 1;
      words += ncap[r];
    }
    DevBuf<uint32_t*> d_nr;
    DevBuf<int64_t> d_nc;
    DevBuf<unsigned long long> nh, nt;
    d_nr.ensure(ss.nsub);
    d_nc.ensure(ss.nsub);
    nh.ensure(ss.nsub);
    nt.ensure(ss.nsub);
    const double t_alloc = now_ms();
    HIPCHK(hipMemcpy(d_nr.p, nring.data(), ss.nsub * sizeof(uint32_t*), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_nc.p, ncap.data(), ss.nsub * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(nh.p, 0, ss.nsub * 8));
    HIPCHK(hipMemset(nt.p, 0, ss.nsub * 8));
    if (!slab_move_raw(e, ss, ss.dir.p, ss.d_ring.p, ss.d_cap.p, ss.tail.p, ss.nsub,
                       std::vector<unsigned long long>(ss.nsub, ~0ull), active, d_nr.p, d_nc.p, nh.p, nt.p, ss.nsub))
      throw Error(SDH_E_CAPACITY, "K_slab: a ring overflowed while growing");
    std::vector<unsigned long long> moved(ss.nsub);
    HIPCHK(hipMemcpy(moved.data(), nh.p, ss.nsub * 8, hipMemcpyDeviceToHost));
    const double t_move = now_ms();
    for (int r = 0; r < ss.nsub; ++r) {
      if (!active[r]) continue;
      ss.free_ring(ss.ring[r], ss.cap[r]);
      ss.ring[r] = nring[r];
      ss.cap[r] = ncap[r];
      ss.h_head[r] = moved[r];
      ss.h_tail[r] = 0;
      ss.h_push0[r] = 0;
    }
    slab_upload_rings(ss);
    HIPCHK(hipMemcpy(ss.head.p, ss.h_head.data(), ss.nsub * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ss.tail.p, ss.h_tail.data(), ss.nsub * 8, hipMemcpyHostToDevice));
    ss.growths += (int64_t)(b1 - b0);
    if (sdh::knob("SDH_SLAB_TRACE"))
      fprintf(stderr, "[sdh] slab grow: %zu rings, %.2f GB: alloc %.1f ms, move %.1f ms, free %.1f ms\n", b1 - b0,
              words * 4e-9, t_alloc - t_start, t_move - t_alloc, now_ms() - t_move);
  }
}

// Room for the next push in every ring. The rings are log-structured: a push appends the entries it
// changes, the old copies die in place. A ring whose free room falls below its live words plus 1.25x
// what it took in the last push is cleaned in place: every block written before that push moves to
// its head (the blocks of the last push are current) -- the oldest 4x the room the next push needs
// (SDH_SLAB_SPAN), mostly dead copies -- once its free room falls below 5x that need (SDH_SLAB_CLEAN_AT):
// a few pushes per cleaning, each a directory pass. A ring below 1.4x (live + headroom) words (SDH_SLAB_GROW_AT) moves
// its live blocks into a fresh buffer of 1.6x that (SDH_SLAB_GROW_TO): the reservation stays
// under 2x the live words, and the cleaning moves (wave-cooperative, nfa_slab.hip) are cheap enough
// to run at most pushes. A push that still overflows is undone and re-run with room for 1.25x its
// demand (re-runs cost time, never matches).
// (C5: cleaning only when a push lacked room never fit in place -- the ring was full by then -- so
// every cleaning reallocated; growing by the ring's span instead of its live words doubled the
// reservation every other step and ran out of HBM.)
// demand: words a failed push tried to take per ring (room for 1.25x that is made instead)
void slab_prepare(sdh_engine* e, sdh_engine::SlabSet& ss, const std::vector<int64_t>* demand = nullptr) {
  const double t_prep = now_ms();
  std::vector<int64_t> need(ss.nsub);
  std::vector<unsigned long long> limit(ss.nsub);
  std::vector<uint8_t> clean(ss.nsub, 0);
  // live words per ring (one pass over the directory)
  std::vector<unsigned long long> live(ss.nsub, 0);
  {
    DevBuf<unsigned long long> acc;
    acc.ensure(ss.nsub);
    HIPCHK(hipMemsetAsync(acc.p, 0, ss.nsub * 8, e->stream));
    HIPCHK(sdh_slab_live_words_ring(ss.dir.p, ss.key_cap * ss.n_groups, ss.n_groups, ss.d_group_ew.p, ss.nsub, acc.p,
                                    e->stream));
    HIPCHK(hipMemcpyAsync(live.data(), acc.p, ss.nsub * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  bool any = false;
  for (int r = 0; r < ss.nsub; ++r) {
    const int64_t alloc = (int64_t)(ss.h_head[r] - ss.h_push0[r]);
    need[r] = std::max<int64_t>(alloc + alloc / 4, 4096);
    if (demand) need[r] = std::max<int64_t>(need[r], (*demand)[r] + (*demand)[r] / 4);
    const int64_t used = (int64_t)(ss.h_head[r] - ss.h_tail[r]);
    // clean once the room falls below SDH_SLAB_CLEAN_AT x the push's need (then the live blocks of
    // the span still fit at the head: the in-place move needs room for them, and a span holds at most
    // SDH_SLAB_SPAN x need live words)
    const double clean_at = sdh::knob("SDH_SLAB_CLEAN_AT") ? atof(sdh::knob("SDH_SLAB_CLEAN_AT")) : 3.0;
    if ((double)(ss.cap[r] - used) >= clean_at * (double)need[r]) continue;
    // the oldest quarter of the ring (at least twice the headroom): mostly dead copies, so the move
    // is small (SDH_SLAB_CLEAN=all: everything before the last push)
    const unsigned long long cur = ss.h_push0[r] > ss.h_tail[r] ? ss.h_push0[r] : ss.h_head[r];
    const bool all = sdh::knob("SDH_SLAB_CLEAN") && !strcmp(sdh::knob("SDH_SLAB_CLEAN"), "all");
    // (the span a push needs, not a fixed share of the ring: every live block in it moves, and the
    // oldest blocks of a ring are not all dead -- a quarter of the ring per push moved 15 % of C5's
    // device time. C5 sweep, CLEAN_AT:SPAN:GROW_TO -> slab_move share of the 24-step run, ms/step,
    // reserved/live: 5:4:1.6 10.0 %, 457, 1.80; 3:2:1.6 7.8 %, 458, 1.95; 3:2:1.5 8.8 %, 447, 1.75;
    // 4:3:1.6 9.0 %, 469, 1.96; 5:8:1.6 30 %, 632; 9:8:1.6 42 %, 822; GROW_TO 2.0 at 5:4 5.9 %, 2.13)
    const double span_x = sdh::knob("SDH_SLAB_SPAN") ? atof(sdh::knob("SDH_SLAB_SPAN")) : 2.0;
    const unsigned long long span = (unsigned long long)std::max<int64_t>((int64_t)(span_x * need[r]), 4096);
    limit[r] = all ? cur : std::min<unsigned long long>(cur, ss.h_tail[r] + span);
    clean[r] = 1;
    any = true;
  }
  std::vector<int> grow;
  std::vector<int64_t> gcap;
  if (any) {
    // (a ring's blocks move within that ring, so rings succeed or fail on their own)
    std::vector<uint8_t> fail;
    (void)slab_move_raw(e, ss, ss.dir.p, ss.d_ring.p, ss.d_cap.p, ss.tail.p, ss.nsub, limit, clean, ss.d_ring.p,
                        ss.d_cap.p, ss.head.p, ss.tail.p, ss.nsub, &fail);
    slab_heads(e, ss);
    for (int r = 0; r < ss.nsub; ++r)
      if (clean[r] && !fail[r]) ss.h_tail[r] = limit[r];
    HIPCHK(hipMemcpy(ss.tail.p, ss.h_tail.data(), ss.nsub * 8, hipMemcpyHostToDevice));
    ++ss.cleanings;
    // a ring below 2x (live + headroom) cannot clean in place for long: a fresh buffer of 2.5x that
    // takes its live blocks (slab_grow compacts as it moves; sized from the live words, not the
    // ring's span, which counts dead blocks: sizing from the span doubled the reservation every
    // other C5 step and ran out of HBM)
    const double grow_at = sdh::knob("SDH_SLAB_GROW_AT") ? atof(sdh::knob("SDH_SLAB_GROW_AT")) : 1.4;
    const double grow_to = sdh::knob("SDH_SLAB_GROW_TO") ? atof(sdh::knob("SDH_SLAB_GROW_TO")) : 1.5;
    for (int r = 0; r < ss.nsub; ++r) {
      if (!clean[r]) continue;
      const int64_t used = (int64_t)(ss.h_head[r] - ss.h_tail[r]);
      const double base = (double)((int64_t)live[r] + need[r]);
      if (!fail[r] && ss.cap[r] - used >= need[r] && (double)ss.cap[r] >= grow_at * base) continue;
      grow.push_back(r);
      gcap.push_back(std::max<int64_t>(ss.cap[r], (int64_t)(grow_to * base)));
    }
  }
  if (sdh::knob("SDH_SLAB_TRACE")) {
    fprintf(stderr, "[sdh] slab prepare: live pass + cleaning %.1f ms\n", now_ms() - t_prep);
    int64_t c = 0, u = 0, nd = 0, g = 0;
    for (int r = 0; r < ss.nsub; ++r) {
      c += ss.cap[r];
      u += (int64_t)(ss.h_head[r] - ss.h_tail[r]);
      nd += need[r];
    }
    for (int64_t x : gcap) g += x;
    fprintf(stderr, "[sdh] slab prepare: %d rings, cap %.2f GB, used %.2f GB, need %.2f GB, demand %d, grow %zu rings to %.2f GB\n",
            ss.nsub, c * 4e-9, u * 4e-9, nd * 4e-9, demand ? 1 : 0, grow.size(), g * 4e-9);
  }
  if (!grow.empty()) slab_grow(e, ss, grow, gcap);
  ss.h_push0 = ss.h_head;
}

// undo this pass's launch of the set (its directory changes; its allocations are dropped)
void slab_rollback(sdh_engine* e, sdh_engine::SlabSet& ss) {
  if (ss.items <= 0) return;
  HIPCHK(sdh_slab_rollback(ss.dir.p, ss.journal.p, ss.journal_idx.p, ss.items, ss.live_bak.p, ss.live.p, e->stream));
  HIPCHK(hipMemcpyAsync(ss.head.p, ss.head_bak.p, ss.nsub * 8, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  ss.items = 0;
  slab_heads(e, ss);
}

int64_t slab_live_partials(sdh_engine* e, const sdh_engine::SlabSet& ss) {
  long long v[256];
  HIPCHK(hipMemcpyAsync(v, ss.live.p, sizeof v, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  int64_t n = 0;
  for (long long x : v) n += x;
  return n;
}

void gen_build(sdh_engine* e, const std::vector<int>& qis) {
  kg::Sizing sz;
  if (e->cfg.gen_pool_states > 0) sz.R = std::min(kg::GMAXPOOL, e->cfg.gen_pool_states);
  if (e->cfg.gen_pool_nodes > 0) sz.N = std::min(kg::GMAXPOOL, e->cfg.gen_pool_nodes);
  if (e->cfg.gen_list_cap > 0) sz.LC = std::min(1 << 16, e->cfg.gen_list_cap);
  e->gsz = sz;
  std::vector<int> gidx(e->lp.q.size(), -1);
  std::vector<KPart> kpart(e->lp.q.size());
  std::vector<char> is_slab(e->lp.q.size(), 0);
  const bool use_part = !(e->cfg.flags & SDH_FLAG_FORCE_GEN) && !sdh::knob("SDH_NO_KPART");
  const bool use_slab = !(e->cfg.flags & SDH_FLAG_FORCE_GEN) && !sdh::knob("SDH_NO_KSLAB");
  for (int qi : qis) {
    try {
      kg::GQuery g = kg::lower_gen(e->lp, qi, sz);
      g.rank = 0;
      if (7 + g.lay.S + g.lay.N > GEN_RING_MARGIN) throw kg::LowerError("match record longer than the ring margin");
      gidx[qi] = (int)e->gq.size();
      e->gq.push_back(g);
      const bool fan = kg::reads_fanout(e->lp, qi);  // fan-out streams run on K_gen (the sweep)
      e->has_fanout |= fan;
      if (use_part && !fan) kpart[qi] = kpart_shape(e->lp, qi, g);
      if (use_slab && !fan && kpart[qi].kind < 0) {
        slab::Shape sh;
        is_slab[qi] = slab::shape_of_query(e->lp, qi, g, &sh, nullptr) ? 1 : 0;
      }
      e->gq_arena.push_back(kpart[qi].kind < 0 && !is_slab[qi]);
      e->has_absent |= g.lay.TQ > 0;
      if (kpart[qi].kind >= 0 || is_slab[qi]) continue;  // K_part / K_slab: no K_gen arena
      e->gB32 = std::max(e->gB32, g.lay.n32);
      e->gB64 = std::max(e->gB64, g.lay.n64);
      e->gHotS = std::max(e->gHotS, g.lay.S);
      if (!g.lay.big) e->gHotNU = std::max(e->gHotNU, g.lay.NU);
    } catch (const kg::LowerError& ex) {
      throw Error(SDH_E_UNSUPPORTED, fmt("query %d: %s", qi, ex.what()));
    }
  }
  if (e->gq.empty()) return;
  // lane_q / group_tmpl rows of one set's members, bucketed by shape (see add_set)
  auto add_groups = [&](const std::vector<int>& members, bool seq_ok) {
    std::vector<std::pair<std::string, std::vector<int>>> shapes;
    for (int qi : members) {
      const kg::GQuery sh = kg::shape_of(e->gq[gidx[qi]]);
      std::string sig((const char*)&sh, sizeof sh);
      auto it = std::find_if(shapes.begin(), shapes.end(), [&](const auto& b) { return b.first == sig; });
      if (it == shapes.end()) shapes.emplace_back(std::move(sig), std::vector<int>{gidx[qi]});
      else it->second.push_back(gidx[qi]);
    }
    int n_groups = 0;
    for (const auto& b : shapes) {
      const int ng = (int)((b.second.size() + 63) / 64);
      const int S = (seq_ok && !(e->cfg.flags & SDH_FLAG_FORCE_GEN)) ? kg::seq_window(e->gq[b.second[0]]) : -1;
      for (int g = 0; g < ng; ++g) {
        e->group_seq.push_back(S > 0 ? S : 0);
        e->group_tmpl.push_back(b.second[0]);
        for (int l = 0; l < 64; ++l) {
          const size_t k = (size_t)g * 64 + l;
          e->lane_q.push_back(k < b.second.size() ? b.second[k] : -1);
        }
      }
      n_groups += ng;
    }
    return n_groups;
  };
  auto route_of = [&](int partition) {
    if ((int)e->routes.size() <= partition) e->routes.resize(partition + 1);
    if (e->routes[partition]) return;
    auto r = std::make_unique<sdh_engine::Route>();
    r->max_keys = e->cfg.gen_max_keys > 0 ? e->cfg.gen_max_keys : (1 << 20);
    int64_t slots = 1;
    while (slots < 2 * r->max_keys) slots <<= 1;
    r->tmask = slots - 1;
    r->tkey.ensure(slots + 1);
    r->tid.ensure(slots + 1);
    std::vector<unsigned long long> init((size_t)slots + 1, 0x8000000000000000ull);
    init[slots] = 0;
    HIPCHK(hipMemcpy(r->tkey.p, init.data(), init.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(r->tid.p, 0xff, (slots + 1) * 4));
    r->n_keys.ensure(1);
    HIPCHK(hipMemset(r->n_keys.p, 0, 4));
    r->key_of_id.ensure(r->max_keys);
    r->track = !e->lp.parts[partition].fanout.empty();
    if (r->track && e->cfg.shard_world > 1)
      throw Error(SDH_E_UNSUPPORTED, "a non-partitioned stream inside a partition with key sharding");
    e->routes[partition] = std::move(r);
  };
  auto add_part_sets = [&](int partition, const std::vector<int>& members) {
    for (int kind = PK_OR; kind <= PK_COUNT; ++kind) {
      std::vector<int> m;
      for (int qi : members)
        if (kpart[qi].kind == kind) m.push_back(qi);
      if (m.empty()) continue;
      route_of(partition);
      auto ps = std::make_unique<sdh_engine::PartSet>();
      ps->partition = partition;
      ps->kind = kind;
      ps->group_base = (int)(e->lane_q.size() / 64);
      ps->n_groups = add_groups(m, false);
      const KPart& k0 = kpart[m[0]];
      ps->sA = k0.sA;
      ps->sB = k0.sB;
      for (int qi : m) {
        ps->cmax = std::max(ps->cmax, kpart[qi].cmax);
        ps->n_e1 = std::max(ps->n_e1, kpart[qi].n_e1);
        ps->n_first = std::max(ps->n_first, kpart[qi].n_first);
        ps->n_last = std::max(ps->n_last, kpart[qi].n_last);
        if (kpart[qi].sA != ps->sA || kpart[qi].sB != ps->sB) throw Error(SDH_E_UNSUPPORTED, "K_part side order");
      }
      ps->ew = kind == PK_COUNT ? 3 + ps->cmax + ps->n_e1 + ps->n_first + ps->n_last : 3;
      ps->cap = kind == PK_COUNT ? 8 : 16;
      if (const char* v = sdh::knob("SDH_KPART_CAP")) ps->cap = std::max(1, atoi(v));
      e->psets.push_back(std::move(ps));
    }
  };
  // K_slab: a partition's distinct-stream patterns in one set (slab.h), groups bucketed by shape
  auto add_slab_set = [&](int partition, const std::vector<int>& members) {
    std::vector<int> m;
    for (int qi : members)
      if (is_slab[qi]) m.push_back(qi);
    if (m.empty()) return;
    route_of(partition);
    auto ss = std::make_unique<sdh_engine::SlabSet>();
    ss->partition = partition;
    ss->group_base = (int)(e->lane_q.size() / 64);
    ss->n_groups = add_groups(m, false);
    std::map<int, int> shape_of_tmpl;
    for (int g = 0; g < ss->n_groups; ++g) {
      const int t = e->group_tmpl[ss->group_base + g];
      auto it = shape_of_tmpl.find(t);
      if (it == shape_of_tmpl.end()) {
        slab::Shape sh;
        std::string why;
        if (!slab::shape_of_query(e->lp, e->gq[t].qid, e->gq[t], &sh, &why))
          throw Error(SDH_E_UNSUPPORTED, "K_slab shape: " + why);
        it = shape_of_tmpl.emplace(t, (int)ss->shapes.size()).first;
        ss->shapes.push_back(sh);
      }
      ss->group_shape.push_back(it->second);
      ss->group_ew.push_back(ss->shapes[it->second].EW);
    }
    const int ns = (int)e->prog.stream_types.size();
    ss->glist.assign(ns, {});
    ss->d_glist.resize(ns);
    for (int g = 0; g < ss->n_groups; ++g)
      for (int st = 0; st < ns && st < kg::GMAXSTREAM; ++st)
        if (ss->shapes[ss->group_shape[g]].proc[st] >= 0) ss->glist[st].push_back(g);
    for (int st = 0; st < ns; ++st) {
      ss->d_glist[st].ensure(std::max<size_t>(1, ss->glist[st].size()));
      if (!ss->glist[st].empty())
        HIPCHK(hipMemcpy(ss->d_glist[st].p, ss->glist[st].data(), ss->glist[st].size() * 4, hipMemcpyHostToDevice));
    }
    ss->d_shapes.ensure(ss->shapes.size());
    HIPCHK(hipMemcpy(ss->d_shapes.p, ss->shapes.data(), ss->shapes.size() * sizeof(slab::Shape), hipMemcpyHostToDevice));
    ss->d_group_shape.ensure(ss->n_groups);
    HIPCHK(hipMemcpy(ss->d_group_shape.p, ss->group_shape.data(), ss->n_groups * 4, hipMemcpyHostToDevice));
    ss->d_group_ew.ensure(ss->n_groups);
    HIPCHK(hipMemcpy(ss->d_group_ew.p, ss->group_ew.data(), ss->n_groups * 4, hipMemcpyHostToDevice));
    if (const char* v = sdh::knob("SDH_SLAB_LDS_WORDS")) ss->lds_words = std::max(64, atoi(v));
    int64_t sub = 1 << 16;  // words per sub-ring; grows on demand (slab_prepare)
    if (const char* v = sdh::knob("SDH_SLAB_SUB_WORDS")) sub = std::max<int64_t>(64, atoll(v));
    slab_init(e, *ss, sub);
    e->ssets.push_back(std::move(ss));
  };
  // sets: the unpartitioned queries, then one per partition; 64 queries per group (wave)
  auto add_set = [&](int partition, const std::vector<int>& members) {
    if (members.empty()) return;
    std::vector<int> gen_m;
    for (int qi : members)
      if (kpart[qi].kind < 0 && !is_slab[qi]) gen_m.push_back(qi);
    if (partition >= 0) add_part_sets(partition, members);
    if (partition >= 0) add_slab_set(partition, members);
    if (gen_m.empty()) return;
    auto gs = std::make_unique<sdh_engine::GenSet>();
    gs->partition = partition;
    gs->group_base = (int)(e->lane_q.size() / 64);
    // one shape per group: members are bucketed by kg::shape_of (first-appearance order) and each
    // bucket is padded to whole groups, so a wave's control flow is its template's. Lane order is
    // free: matches are ordered by (seq, out_rank, emission index) in the device match table.
    gs->n_groups = add_groups(gen_m, partition < 0);
    const size_t per_block32 = (size_t)e->gB32 * 64, per_block64 = (size_t)e->gB64 * 64;
    if (partition < 0) {
      gs->a32.ensure(per_block32 * gs->n_groups);
      gs->a64.ensure(per_block64 * gs->n_groups);
      HIPCHK(hipMemset(gs->a32.p, 0, per_block32 * gs->n_groups * 4));
      HIPCHK(hipMemset(gs->a64.p, 0, per_block64 * gs->n_groups * 8));
    } else {
      route_of(partition);
      gs->key_cap = 0;
    }
    e->gsets.push_back(std::move(gs));
  };
  std::vector<int> top;
  for (int qi : qis)
    if (e->lp.q[qi].partition < 0) top.push_back(qi);
  add_set(-1, top);
  for (int pi = 0; pi < (int)e->lp.parts.size(); ++pi) {
    // lanes in definition order, not the partition's receiver order (LPart::queries is the
    // metaQueryRuntimeMap order, which scatters a family's neighbouring queries): lane order is free
    // (the match table orders rows by rank), and neighbouring definitions share a wave's control
    // flow more often (C3: 20.9 ms/step in receiver order)
    std::vector<int> m;
    for (int qi : e->lp.parts[pi].queries)
      if (gidx[qi] >= 0) m.push_back(qi);
    std::sort(m.begin(), m.end());
    add_set(pi, m);
  }
  e->d_gq.ensure(e->gq.size());
  HIPCHK(hipMemcpy(e->d_gq.p, e->gq.data(), e->gq.size() * sizeof(kg::GQuery), hipMemcpyHostToDevice));
  // the groups' lane-constant table (kg::LaneConsts): [group][slot][64], slot 0 query id, 1 within,
  // 2 + k the k-th CONST instruction of the group's shape; idle lanes repeat the template's values
  {
    const size_t n_groups = e->group_tmpl.size();
    int slots = kg::LC_FIRST;
    std::vector<std::vector<int>> pcs(n_groups);
    for (size_t g = 0; g < n_groups; ++g) {
      const kg::GQuery& t = e->gq[e->group_tmpl[g]];
      for (int pc = 0; pc < t.n_code; ++pc)
        if (t.code[pc].op == kg::OP_CONST) pcs[g].push_back(pc);
      slots = std::max(slots, kg::LC_FIRST + (int)pcs[g].size());
    }
    std::vector<int64_t> lc(std::max<size_t>(1, n_groups * slots * 64), 0);
    for (size_t g = 0; g < n_groups; ++g)
      for (int l = 0; l < 64; ++l) {
        const int qi = e->lane_q[g * 64 + l];
        const kg::GQuery& x = e->gq[qi >= 0 ? qi : e->group_tmpl[g]];
        int64_t* row = lc.data() + g * slots * 64 + l;
        row[kg::LC_QID * 64] = x.qid;
        row[kg::LC_WITHIN * 64] = x.within;
        for (size_t k = 0; k < pcs[g].size(); ++k) row[(kg::LC_FIRST + k) * 64] = x.code[pcs[g][k]].imm;
      }
    e->lc_slots = slots;
    e->d_lconst.ensure(lc.size());
    HIPCHK(hipMemcpy(e->d_lconst.p, lc.data(), lc.size() * 8, hipMemcpyHostToDevice));
  }
  e->d_lane_q.ensure(e->lane_q.size());
  HIPCHK(hipMemcpy(e->d_lane_q.p, e->lane_q.data(), e->lane_q.size() * 4, hipMemcpyHostToDevice));
  e->seq_tail.resize(e->prog.stream_types.size());
  e->seq_tail_len.assign(e->prog.stream_types.size(), 0);
  for (auto& t : e->seq_tail) {
    t.ensure(SEQ_TMAX * SEQ_TW);
    HIPCHK(hipMemset(t.p, 0, SEQ_TMAX * SEQ_TW * 8));
  }
  e->d_glists.resize(e->prog.stream_types.size() + 1);
  spec_build(e);
  e->d_group_tmpl.ensure(e->group_tmpl.size());
  HIPCHK(hipMemcpy(e->d_group_tmpl.p, e->group_tmpl.data(), e->group_tmpl.size() * 4, hipMemcpyHostToDevice));
  e->g_out_next.ensure(1);
  e->g_nrec.ensure(1);
  e->d_perr.ensure(std::max<size_t>(1, e->psets.size()) * 4);
  e->d_serr.ensure(std::max<size_t>(1, e->ssets.size()) * 4);
}

// grow a partition set's instance arena to hold `keys` keys (blocks are key-major: a prefix copy)
void gen_grow(sdh_engine* e, sdh_engine::GenSet& gs, int64_t keys) {
  if (keys <= gs.key_cap) return;
  int64_t cap = std::max<int64_t>(64, gs.key_cap);
  while (cap < keys) cap *= 2;
  const size_t b32 = (size_t)e->gB32 * 64 * gs.n_groups, b64 = (size_t)e->gB64 * 64 * gs.n_groups;
  DevBuf<int32_t> n32;
  DevBuf<int64_t> n64;
  n32.ensure(b32 * cap);
  n64.ensure(b64 * cap);
  HIPCHK(hipMemsetAsync(n32.p, 0, b32 * cap * 4, e->stream));
  HIPCHK(hipMemsetAsync(n64.p, 0, b64 * cap * 8, e->stream));
  if (gs.key_cap > 0) {
    HIPCHK(hipMemcpyAsync(n32.p, gs.a32.p, b32 * gs.key_cap * 4, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(n64.p, gs.a64.p, b64 * gs.key_cap * 8, hipMemcpyDeviceToDevice, e->stream));
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  std::swap(gs.a32.p, n32.p);
  std::swap(gs.a32.n, n32.n);
  std::swap(gs.a64.p, n64.p);
  std::swap(gs.a64.n, n64.n);
  gs.key_cap = cap;
}


// K_gen pools and lists at a new sizing: every query's layout is recomputed (make_layout) and each
// set's arenas are re-laid on the device (gen_remap_kernel; remap = false: zeroed, the caller
// overwrites them). Pools only grow between pushes, so the indices the arenas hold stay valid.
void gen_relayout(sdh_engine* e, const kg::Sizing& sz, bool remap) {
  if (7 + kg::GMAXS + sz.N > GEN_RING_MARGIN) throw Error(SDH_E_CAPACITY, "K_gen node pool beyond the match-record limit");
  std::vector<kg::GLayout> oldL(e->gq.size()), newL(e->gq.size());
  int b32 = 1, b64 = 1, hot_nu = 1;
  for (size_t i = 0; i < e->gq.size(); ++i) {
    kg::GQuery& g = e->gq[i];
    oldL[i] = g.lay;
    kg::make_layout(g.lay, g.lay.S, sz.R, sz.N, sz.LC, g.lay.NA, g.lay.v32 != 0, g.lay.TQ > 0 ? sz.LC : 0);
    newL[i] = g.lay;
    if (!e->gq_arena[i]) continue;
    b32 = std::max(b32, g.lay.n32);
    b64 = std::max(b64, g.lay.n64);
    if (!g.lay.big) hot_nu = std::max(hot_nu, g.lay.NU);
  }
  DevBuf<kg::GLayout> dOld, dNew;
  dOld.ensure(oldL.size());
  dNew.ensure(newL.size());
  HIPCHK(hipMemcpy(dOld.p, oldL.data(), oldL.size() * sizeof(kg::GLayout), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dNew.p, newL.data(), newL.size() * sizeof(kg::GLayout), hipMemcpyHostToDevice));
  for (auto& up : e->gsets) {
    auto& gs = *up;
    const int64_t blocks = gs.partition < 0 ? gs.n_groups : gs.key_cap * gs.n_groups;
    DevBuf<int32_t> n32;
    DevBuf<int64_t> n64;
    n32.ensure(std::max<size_t>(1, (size_t)blocks * b32 * 64));
    n64.ensure(std::max<size_t>(1, (size_t)blocks * b64 * 64));
    HIPCHK(hipMemsetAsync(n32.p, 0, n32.n * 4, e->stream));
    HIPCHK(hipMemsetAsync(n64.p, 0, n64.n * 8, e->stream));
    if (remap)
      HIPCHK(sdh_gen_remap(e->d_lane_q.p, gs.group_base, gs.n_groups, blocks, dOld.p, dNew.p, gs.a32.p, gs.a64.p,
                           e->gB32, e->gB64, n32.p, n64.p, b32, b64, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    std::swap(gs.a32.p, n32.p);
    std::swap(gs.a32.n, n32.n);
    std::swap(gs.a64.p, n64.p);
    std::swap(gs.a64.n, n64.n);
  }
  e->gB32 = b32;
  e->gB64 = b64;
  e->gHotNU = hot_nu;
  e->gsz = sz;
  HIPCHK(hipMemcpy(e->d_gq.p, e->gq.data(), e->gq.size() * sizeof(kg::GQuery), hipMemcpyHostToDevice));
}

// the sizing after a K_gen capacity failure of kinds `capk` (kg::CAP_*): each limit hit doubles
bool gen_grown_sizing(const sdh_engine* e, int capk, kg::Sizing* out) {
  kg::Sizing sz = e->gsz;
  if (capk & kg::CAP_FIXED) return false;
  if (capk & kg::CAP_STATES) sz.R = std::min(kg::GMAXPOOL, 2 * sz.R);
  if (capk & kg::CAP_NODES) sz.N = std::min(kg::GMAXPOOL, 2 * sz.N);
  if (capk & kg::CAP_LIST) sz.LC = std::min(1 << 16, 2 * sz.LC);
  if (sz.R == e->gsz.R && sz.N == e->gsz.N && sz.LC == e->gsz.LC) return false;
  *out = sz;
  return true;
}


// Exact re-runs (the reference never drops a match): just before a K_gen launch modifies a set's
// arena blocks, they are journaled (gen_journal_kernel); a pass whose match output, pools, K_part
// tables or K_slab space overflowed is undone by copying them back, and re-run at the grown size.
// The journal holds the blocks of this pass only -- the set's groups (unpartitioned), the pushed
// keys' blocks (partitions), every known key's (a timer sweep) -- so its cost scales with the push,
// not with the total state. mode / glist / seg_kid: as gen_journal_kernel.
void gen_journal(sdh_engine* e, sdh_engine::GenSet& gs, int mode, const int32_t* glist, const uint32_t* seg_kid,
                 int64_t slots) {
  gs.jn = 0;
  if (!e->g_journal || slots <= 0) return;
  const size_t b32 = (size_t)e->gB32 * 64, b64 = (size_t)e->gB64 * 64;
  gs.j32.ensure(b32 * slots);
  gs.j64.ensure(b64 * slots);
  gs.jidx.ensure((size_t)slots);
  HIPCHK(sdh_gen_journal(gs.a32.p, gs.a64.p, e->gB32, e->gB64, mode, glist, seg_kid, gs.n_groups, slots, gs.j32.p,
                         gs.j64.p, gs.jidx.p, 0, e->stream));
  gs.jn = slots;
}

void gen_restore_journal(sdh_engine* e) {
  for (auto& up : e->gsets) {
    auto& gs = *up;
    if (gs.jn > 0)
      HIPCHK(sdh_gen_journal(gs.a32.p, gs.a64.p, e->gB32, e->gB64, 0, nullptr, nullptr, gs.n_groups, gs.jn, gs.j32.p,
                             gs.j64.p, gs.jidx.p, 1, e->stream));
    gs.jn = 0;
  }
  HIPCHK(hipStreamSynchronize(e->stream));
}

// Upper bound of the journal bytes a push of n events over `stream` needs; do_push splits a batch
// whose bound does not fit a third of free HBM
double gen_journal_bound(sdh_engine* e, int64_t n) {
  double blocks = 0;
  for (auto& up : e->gsets) {
    auto& gs = *up;
    if (gs.partition < 0) {
      blocks += gs.n_groups;
      continue;
    }
    bool timed = false;
    for (int g = 0; g < gs.n_groups; ++g) timed |= e->gq[e->group_tmpl[gs.group_base + g]].lay.TQ > 0;
    blocks += (double)gs.n_groups * (double)(timed ? gs.key_cap + n : n);
  }
  return blocks * ((double)e->gB32 * 64 * 4 + (double)e->gB64 * 64 * 8);
}

// one K_gen step for every set fed by `stream`
sdh::GenLaunch gen_launch_base(sdh_engine* e, const sdh_engine::GenSet& gs, const StreamBatch& B, bool write) {
  sdh::GenLaunch L{};
  L.queries = e->d_gq.p;
  L.lane_q = e->d_lane_q.p;
  L.group_tmpl = e->d_group_tmpl.p;
  L.b = B;
  L.groups = gs.n_groups;
  L.group_base = gs.group_base;
  L.B32 = e->gB32;
  L.B64 = e->gB64;
  L.hot_s = e->gHotS;
  L.hot_nu = e->gHotNU;
  L.out = e->g_out.p;
  L.out_cap = e->g_out_cap;
  L.out_next = e->g_out_next.p;
  L.err = e->d_err.p;
  L.rec_count = e->g_nrec.p;
  L.rec_off = e->g_rec_off.p;
  L.rec_cap = e->g_out_cap / NREC_MIN_WORDS + 1;
  L.rec_next = e->g_rec_next.p;
  L.write_records = write ? 1 : 2;
  L.start_ts = e->start_ts;
  L.advance_to = e->advance_to;
  L.timer_seq = e->seq + B.n;
  L.playback = (e->cfg.flags & SDH_FLAG_PLAYBACK) ? 1 : 0;
  L.no_timers = e->ck.active ? 1 : 0;
  L.xcd = e->xcd;
  return L;
}

// K_part state: room for `keys` keys (new keys' blocks start empty: n = 0, buffer 0)
void part_grow(sdh_engine* e, sdh_engine::PartSet& ps, int64_t keys) {
  if (keys <= ps.key_cap) return;
  int64_t cap = std::max<int64_t>(64, ps.key_cap);
  while (cap < keys) cap *= 2;
  const size_t per_key = (size_t)ps.n_groups * ps.bw() * 64;  // int64 words per key and buffer
  DevBuf<int64_t> nst;
  DevBuf<int32_t> ncur, nnxt;
  nst.ensure(2 * per_key * cap);
  ncur.ensure(cap);
  nnxt.ensure(cap);
  HIPCHK(hipMemsetAsync(nst.p, 0, 2 * per_key * cap * 8, e->stream));
  HIPCHK(hipMemsetAsync(ncur.p, 0, cap * 4, e->stream));
  if (ps.key_cap > 0)
    for (int b = 0; b < 2; ++b)
      HIPCHK(hipMemcpyAsync(nst.p + b * per_key * cap, ps.st.p + b * per_key * ps.key_cap, per_key * ps.key_cap * 8,
                            hipMemcpyDeviceToDevice, e->stream));
  if (ps.key_cap > 0) HIPCHK(hipMemcpyAsync(ncur.p, ps.cur.p, ps.key_cap * 4, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::swap(ps.st.p, nst.p);
  std::swap(ps.st.n, nst.n);
  std::swap(ps.cur.p, ncur.p);
  std::swap(ps.cur.n, ncur.n);
  std::swap(ps.nxt.p, nnxt.p);
  std::swap(ps.nxt.n, nnxt.n);
  ps.key_cap = cap;
}

// K_part entry capacity x2: every block keeps its header and entries at the same word offsets
void part_grow_cap(sdh_engine* e, sdh_engine::PartSet& ps) {
  const int64_t blocks = 2 * ps.key_cap * ps.n_groups, obw = ps.bw();
  ps.cap *= 2;
  if (ps.key_cap == 0) return;
  const int64_t nbw = ps.bw();
  DevBuf<int64_t> nst;
  nst.ensure((size_t)(blocks * nbw * 64));
  HIPCHK(hipMemsetAsync(nst.p, 0, (size_t)blocks * nbw * 64 * 8, e->stream));
  HIPCHK(hipMemcpy2DAsync(nst.p, (size_t)nbw * 64 * 8, ps.st.p, (size_t)obw * 64 * 8, (size_t)obw * 64 * 8, (size_t)blocks,
                          hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::swap(ps.st.p, nst.p);
  std::swap(ps.st.n, nst.n);
}

// One pass of every K_gen / K_seq launch of a push over `stream` (partition routing, arena growth,
// kernels, the event-chunk copy-backs). Returns whether anything ran; *tail_new_len (>= 0) is the
// stream's K_seq tail length once the pass is accepted.
bool gen_pass(sdh_engine* e, int stream, const StreamBatch& B, bool write, double* bytes_out, int32_t* tail_new_len) {
  const int64_t n = B.n;
  int64_t ev_bytes = 8;
  for (int a = 0; a < B.n_attr; ++a) ev_bytes += B.width[a];
  double bytes = 0;
  bool any = false;
  e->stats.last_gen_items = 0;
  e->stats.last_seq_items = 0;
  e->stats.last_part_items = 0;
  for (auto& up : e->gsets) {
    auto& gs = *up;
    if (gs.partition >= 0) continue;  // partitions below
    sdh::GenLaunch L = gen_launch_base(e, gs, B, write);
    {
      // groups reading this stream: windowed sequences go to K_seq, the rest to K_gen
      std::vector<int32_t> seq_rows, gen_groups;
      int seqS = 1;
      for (int g = 0; g < gs.n_groups; ++g) {
        const kg::GQuery& tq = e->gq[e->group_tmpl[gs.group_base + g]];
        const bool timed = tq.lay.TQ > 0;  // absent states: time passes on every push and advance
        if (n == 0 ? !timed : (tq.recv_n[stream] == 0 && !timed)) continue;
        if (e->group_seq[gs.group_base + g] > 0) {
          seq_rows.push_back(gs.group_base + g);
          seqS = std::max(seqS, e->group_seq[gs.group_base + g]);
        } else {
          gen_groups.push_back(g);
        }
      }
      if (seq_rows.empty() && gen_groups.empty()) continue;
      // the lists depend on the stream only: uploaded once, before any kernel reads them
      // (one cached list per stream, and one more for time advances: B.n == 0)
      auto& gl = e->d_glists[n == 0 ? e->prog.stream_types.size() : (size_t)stream];
      if (!gl.p) {
        gl.ensure(std::max<size_t>(1, seq_rows.size() + gen_groups.size()));
        std::vector<int32_t> both(seq_rows);
        both.insert(both.end(), gen_groups.begin(), gen_groups.end());
        if (!both.empty()) HIPCHK(hipMemcpy(gl.p, both.data(), both.size() * 4, hipMemcpyHostToDevice));
      }
      // K_seq: one launch per shape (rows of one shape are contiguous), its compiled kernel if any
      for (size_t r0 = 0, r1 = 0; r0 < seq_rows.size(); r0 = r1) {
        const int tmpl = e->group_tmpl[seq_rows[r0]];
        for (r1 = r0 + 1; r1 < seq_rows.size() && e->group_tmpl[seq_rows[r1]] == tmpl;) ++r1;
        const int nrows = (int)(r1 - r0);
        sdh::SeqLaunch Q{};
        Q.xcd = e->xcd;
        Q.queries = e->d_gq.p;
        Q.lane_q = e->d_lane_q.p;
        Q.group_tmpl = e->d_group_tmpl.p;
        Q.glist = gl.p + r0;
        Q.n_glist = nrows;
        Q.b = B;
        Q.tail = e->seq_tail[stream].p;
        Q.tail_len = e->seq_tail_len[stream];
        Q.write_records = write ? 1 : 2;
        Q.out = e->g_out.p;
        Q.out_cap = e->g_out_cap;
        Q.out_next = e->g_out_next.p;
        Q.rec_count = e->g_nrec.p;
        Q.rec_off = e->g_rec_off.p;
        Q.rec_cap = e->g_out_cap / NREC_MIN_WORDS + 1;
        Q.rec_next = e->g_rec_next.p;
        Q.err = e->d_err.p;
        const int64_t starts = n + Q.tail_len;
        // items per launch: many short chunks balance the chunks' uneven match density (C4 sweep,
        // tools/sweep_seq.sh: 4,096 items 25.2 ms/step, 8,192 19.8, 16,384 17.2, 32,768 16.2, 65,536
        // 15.8, 131,072 15.5)
        const int64_t seq_waves = sdh::knob("SDH_SEQ_WAVES") ? atoll(sdh::knob("SDH_SEQ_WAVES")) : 131072;
        const int64_t target = std::max<int64_t>(1, seq_waves / (int64_t)nrows);
        int64_t clen = std::max<int64_t>(256, (starts + target - 1) / target);
        clen = (clen + 63) / 64 * 64;  // whole LDS tiles
        Q.chunk_len = clen;
        Q.n_chunks = (int32_t)((starts + clen - 1) / clen);
        auto sp = e->seq_spec.find(tmpl);
        if (sp != e->seq_spec.end()) {
          void* args[] = {&Q};
          const int64_t items = (int64_t)Q.n_glist * Q.n_chunks;
          HIPCHK(hipModuleLaunchKernel(sp->second, (unsigned)(Q.xcd ? (items + 7) & ~7ll : items), 1, 1, 64, 1, 1, 0,
                                       e->stream, args, nullptr));
        } else {
          HIPCHK(sdh_launch_seq(&Q, e->stream));
        }
        *tail_new_len = (int32_t)std::min<int64_t>(SEQ_TMAX, Q.tail_len + n);
        e->stats.last_seq_items += (int64_t)Q.n_glist * Q.n_chunks;
        any = true;
        bytes += (double)n * ev_bytes * nrows;  // every group stages the batch once
      }
      if (gen_groups.empty()) continue;
      L.glist = gl.p + seq_rows.size();
      L.n_glist = (int32_t)gen_groups.size();
      L.a32 = gs.a32.p;
      L.a64 = gs.a64.p;
      // event chunks when every group's shape has a bounded look-back (kg::seq_lookback): chunk
      // c > 0 rebuilds its instances from a few replayed events, so one set fills the chip
      int look = 0;
      for (int g : gen_groups) {
        const int lb = kg::seq_lookback(e->gq[e->group_tmpl[gs.group_base + g]]);
        look = lb < 0 ? -1 : std::max(look, lb);
        if (look < 0) break;
      }
      int64_t C = 1, clen = n;
      if (look >= 0 && n > 0) {
        int64_t minlen = std::max<int64_t>(256, 8 * look);
        if (const char* v = sdh::knob("SDH_GEN_CHUNK_LEN")) minlen = std::max<int64_t>(std::max(1, look), atoll(v));
        const int64_t target = std::max<int64_t>(1, 8192 / (int64_t)gen_groups.size());
        C = std::max<int64_t>(1, std::min<int64_t>((n + minlen - 1) / minlen, target));
        clen = (n + C - 1) / C;
        C = (n + clen - 1) / clen;
      }
      L.n_items = (int32_t)(C * gen_groups.size());
      L.ev_chunks = (int32_t)C;
      L.chunk_len = clen;
      const size_t blk32 = (size_t)e->gB32 * 64, blk64 = (size_t)e->gB64 * 64;
      if (C > 1) {
        gs.s32.ensure(blk32 * gs.n_groups * (C - 1));  // (indexed by set-relative group)
        gs.s64.ensure(blk64 * gs.n_groups * (C - 1));
        L.s32 = gs.s32.p;
        L.s64 = gs.s64.p;
      }
      gen_journal(e, gs, 0, L.glist, nullptr, (int64_t)gen_groups.size());
      HIPCHK(sdh_launch_gen(&L, e->stream));
      e->stats.last_gen_items += L.n_items;
      if (C > 1) {  // the last chunk's instances are the set's state after this batch
        for (int g : gen_groups) {
          const size_t sb = (size_t)(C - 2) * gs.n_groups + g;
          HIPCHK(hipMemcpyAsync(gs.a32.p + g * blk32, gs.s32.p + sb * blk32, blk32 * 4, hipMemcpyDeviceToDevice,
                                e->stream));
          HIPCHK(hipMemcpyAsync(gs.a64.p + g * blk64, gs.s64.p + sb * blk64, blk64 * 8, hipMemcpyDeviceToDevice,
                                e->stream));
        }
      }
      any = true;
      bytes += (double)n * ev_bytes * gen_groups.size();  // every group streams the batch once
      continue;
    }
  }
  // partitions: route the batch once (dense key ids, events grouped by key), then run the
  // partition's K_gen set and its K_part sets over the same segments. A K_gen set with absent states
  // runs as a timer sweep instead: every known key's clone walks the whole batch (time passes for it
  // at every event of any key or stream) and processes its own key's events; a time advance, or a
  // batch of a stream the partition does not key, sweeps with no own events
  for (int pi = 0; pi < (int)e->routes.size(); ++pi) {
    if (!e->routes[pi]) continue;
    auto& rt = *e->routes[pi];
    const kg::LPart& pd = e->lp.parts[pi];
    int attr = -1;
    for (const auto& k : pd.keys)
      if (k.stream == stream) attr = (int)k.code[0].imm;
    sdh_engine::GenSet* gsp = nullptr;
    for (auto& up : e->gsets)
      if (up->partition == pi) gsp = up.get();
    bool timed = false;
    if (gsp)
      for (int g = 0; g < gsp->n_groups; ++g) timed |= e->gq[e->group_tmpl[gsp->group_base + g]].lay.TQ > 0;
    // an ordered batch takes the indexed sweep (each key walks its own events; its timers fire at the
    // first event whose time reaches them, found by binary search), else every key walks the batch
    auto ordered = [&]() {
      if (n <= 0 || sdh::knob("SDH_NO_TIMER_INDEX")) return false;
      e->t_pm.ensure((size_t)n);
      e->t_flag.ensure(1);
      e->t_temp.ensure(sdh_prefix_max_temp_bytes(n));
      HIPCHK(sdh_prefix_max(B.ts, n, e->t_pm.p, e->t_flag.p, e->t_temp.p, e->t_temp.n, e->stream));
      int32_t un = 1;
      HIPCHK(hipMemcpyAsync(&un, e->t_flag.p, 4, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      return un == 0;
    };
    auto sweep = [&](const uint32_t* ev_kid, int64_t n_keys, bool indexed = false, bool own = false,
                     const int32_t* fan_pos = nullptr) {
      auto& gs = *gsp;
      sdh::GenLaunch L = gen_launch_base(e, gs, B, write);
      L.a32 = gs.a32.p;
      L.a64 = gs.a64.p;
      L.key_of_id = rt.key_of_id.p;
      L.sweep = 1;
      L.ev_kid = ev_kid;
      L.n_keys = n_keys;
      L.fan_pos = fan_pos;
      if (indexed) {
        L.pm = e->t_pm.p;
        if (own) {  // the keys' own events: the routed segments
          e->t_kseg.ensure((size_t)std::max<int64_t>(1, n_keys));
          HIPCHK(sdh_key_segments(e->r_uniq.p, e->r_nruns.p, n, n_keys, e->t_kseg.p, e->stream));
          L.kseg = e->t_kseg.p;
          L.seg_begin = e->r_off.p;
          L.seg_len = e->r_cnt.p;
          L.ev_idx = e->r_idx_s.p;
        }
      }
      L.n_items = (int32_t)(n_keys * gs.n_groups);
      gen_journal(e, gs, 2, nullptr, nullptr, (int64_t)L.n_items);
      if (L.n_items > 0) HIPCHK(sdh_launch_gen(&L, e->stream));
      e->stats.last_gen_items += L.n_items;
      any = true;
      // indexed: each key reads its own events and binary-searches pm per timer stop
      bytes += (double)n * ev_bytes * gs.n_groups * (indexed ? 1.0 : (double)n_keys);
    };
    // a stream the partition does not key reaches every known key's clones (PartitionStreamReceiver
    // .send(ComplexEvent):277-281), ordered by the junction map (fan_positions)
    const kg::LFanOut* fo = n > 0 && attr < 0 && gsp && gsp->n_groups > 0 ? pd.fan(stream) : nullptr;
    if (n == 0 || attr < 0) {
      if (timed || fo) {
        int32_t nk = 0;
        HIPCHK(hipMemcpyAsync(&nk, rt.n_keys.p, 4, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        const int64_t nks = std::min<int64_t>(nk, gsp->key_cap);
        if (fo) sweep(nullptr, nks, false, false, fan_positions(e, rt, *fo, nks));
        else sweep(nullptr, nks, ordered(), false);
      }
      continue;
    }
    bool reads = (gsp && gsp->n_groups > 0) || rt.track;  // (fan-out: every key's creation counts)
    for (auto& ps : e->psets)
      if (ps->partition == pi) reads = true;
    for (auto& ss : e->ssets)
      if (ss->partition == pi && !ss->glist[stream].empty()) reads = true;
    if (!reads) continue;
    const int type = e->lp.stream_types[stream][attr];
    e->r_key.ensure(n);
    e->r_kid.ensure(n);
    e->r_kid_s.ensure(n);
    e->r_uniq.ensure(n);
    e->r_idx.ensure(n);
    e->r_idx_s.ensure(n);
    e->r_cnt.ensure(n);
    e->r_off.ensure(n);
    e->r_nruns.ensure(1);
    const size_t tb = sdh_route_temp_bytes(n);
    e->r_temp.ensure(tb);
    HIPCHK(sdh_route_partition(&B, attr, type, rt.tkey.p, rt.tid.p, rt.tmask, rt.n_keys.p, rt.key_of_id.p,
                               rt.max_keys, e->r_key.p, e->r_kid.p, e->r_kid_s.p, e->r_idx.p, e->r_idx_s.p,
                               e->r_uniq.p, e->r_cnt.p, e->r_off.p, e->r_nruns.p, e->r_temp.p, e->r_temp.n,
                               e->d_err.p + 3, e->cfg.shard_rank, e->cfg.shard_world, e->stream));
    int32_t hv[2];
    HIPCHK(hipMemcpyAsync(&hv[0], rt.n_keys.p, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&hv[1], e->r_nruns.p, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (hv[0] > rt.max_keys) throw Error(SDH_E_CAPACITY, "more partition keys than gen_max_keys");
    // events this engine keeps (null keys and, with key sharding, other ranks' keys sort last)
    if (hv[1] > 0) {
      uint32_t last_kid = 0;
      int32_t last_cnt = 0;
      HIPCHK(hipMemcpyAsync(&last_kid, e->r_uniq.p + hv[1] - 1, 4, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipMemcpyAsync(&last_cnt, e->r_cnt.p + hv[1] - 1, 4, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      if ((int)e->part_kept.size() <= pi) e->part_kept.resize(pi + 1, 0);
      e->part_kept[pi] = n - (last_kid == 0xFFFFFFFFu ? last_cnt : 0);
    }
    if (rt.track && hv[0] > rt.nk_seen)
      track_new_keys(e, rt, hv[0], hv[1],
                     type == kg::T_BOOL ? 1 : type == kg::T_STRING ? 2 : type == kg::T_FLOAT ? 3 : type == kg::T_DOUBLE ? 4 : 0);
    // routing (key column read, key/kid/idx written and sorted)
    bytes += (double)n * (8 + 8 + 4 + 4 + 2 * (4 + 4) + 3 * 4);
    if (gsp && gsp->n_groups > 0 && timed) {
      gen_grow(e, *gsp, hv[0]);
      const bool ix = ordered();
      sweep(e->r_kid.p, hv[0], ix, true);
    } else if (gsp && gsp->n_groups > 0) {
      auto& gs = *gsp;
      gen_grow(e, gs, hv[0]);
      sdh::GenLaunch L = gen_launch_base(e, gs, B, write);
      L.a32 = gs.a32.p;
      L.a64 = gs.a64.p;
      L.seg_begin = e->r_off.p;
      L.seg_len = e->r_cnt.p;
      L.seg_kid = e->r_uniq.p;
      L.key_of_id = rt.key_of_id.p;
      L.ev_idx = e->r_idx_s.p;
      L.n_items = hv[1] * gs.n_groups;
      gen_journal(e, gs, 1, nullptr, e->r_uniq.p, (int64_t)L.n_items);
      HIPCHK(sdh_launch_gen(&L, e->stream));
      e->stats.last_gen_items += L.n_items;
      any = true;
      bytes += (double)n * ev_bytes * gs.n_groups;  // every group streams its keys' events
    }
    // K_part reads each key's events as one contiguous run of a key-ordered copy of the batch (the
    // routing sort's order) instead of gathering them from the batch
    sdh::StreamBatch SB{};
    bool sorted = false;
    for (size_t si = 0; si < e->psets.size(); ++si) {
      auto& ps = *e->psets[si];
      if (ps.partition != pi) continue;
      part_grow(e, ps, hv[0]);
      if (!sorted && !sdh::knob("SDH_KPART_GATHER")) {
        e->sb_buf.ensure(sdh_sorted_batch_bytes(&B));
        HIPCHK(sdh_sort_batch(&B, e->r_idx_s.p, e->sb_buf.p, &SB, e->stream));
        sorted = true;
      }
      sdh::PartLaunch P{};
      P.sorted = sorted ? 1 : 0;
      P.xcd = e->xcd;
      P.lconst = e->d_lconst.p;
      P.lc_slots = e->lc_slots;
      P.queries = e->d_gq.p;
      P.lane_q = e->d_lane_q.p;
      P.group_tmpl = e->d_group_tmpl.p;
      P.b = sorted ? SB : B;
      P.seg_begin = e->r_off.p;
      P.seg_len = e->r_cnt.p;
      P.seg_kid = e->r_uniq.p;
      P.key_of_id = rt.key_of_id.p;
      P.ev_idx = e->r_idx_s.p;
      P.groups = ps.n_groups;
      P.group_base = ps.group_base;
      P.kind = ps.kind;
      P.cap = ps.cap;
      P.ew = ps.ew;
      P.sA = ps.sA;
      P.sB = ps.sB;
      P.cmax = ps.cmax;
      P.n_e1 = ps.n_e1;
      P.n_first = ps.n_first;
      P.n_last = ps.n_last;
      P.st = ps.st.p;
      P.blocks = ps.key_cap * ps.n_groups;
      P.cur = ps.cur.p;
      P.nxt = ps.nxt.p;
      P.out = e->g_out.p;
      P.out_cap = e->g_out_cap;
      P.out_next = e->g_out_next.p;
      P.rec_count = e->g_nrec.p;
      P.rec_off = e->g_rec_off.p;
      P.rec_cap = e->g_out_cap / NREC_MIN_WORDS + 1;
      P.rec_next = e->g_rec_next.p;
      P.write_records = write ? 1 : 2;
      if (!write && sdh::knob("SDH_DEBUG_COUNT_ONLY")) P.write_records = 0;  // (measurement experiments)
      P.err = e->d_perr.p + 4 * si;
      const bool prof = sdh::knob("SDH_PART_PROF") != nullptr;
      if (prof) {
        e->d_pprof.ensure(8);
        HIPCHK(hipMemsetAsync(e->d_pprof.p, 0, 8 * 8, e->stream));
        P.prof = e->d_pprof.p;
      }
      // the per-key buffer selector of untouched keys carries over
      HIPCHK(hipMemcpyAsync(ps.nxt.p, ps.cur.p, (size_t)ps.key_cap * 4, hipMemcpyDeviceToDevice, e->stream));
      // one launch per shape (its groups are contiguous), the shape-compiled kernel if there is one
      for (int g0 = 0, g1 = 0; g0 < ps.n_groups; g0 = g1) {
        const int tmpl = e->group_tmpl[ps.group_base + g0];
        for (g1 = g0 + 1; g1 < ps.n_groups && e->group_tmpl[ps.group_base + g1] == tmpl;) ++g1;
        P.g0 = g0;
        P.gn = g1 - g0;
        P.n_items = hv[1] * P.gn;
        auto sp = ps.spec.find(tmpl);
        if (sp != ps.spec.end()) {
          if (P.n_items > 0) {
            void* args[] = {&P};
            HIPCHK(hipModuleLaunchKernel(sp->second, (unsigned)(P.xcd ? (P.n_items + 7) & ~7 : P.n_items), 1, 1, 64, 1,
                                         1, 0, e->stream, args, nullptr));
          }
        } else {
          HIPCHK(sdh_launch_part(&P, e->stream));
        }
        e->stats.last_part_items += P.n_items;
      }
      if (prof) {  // per-phase clocks of this set's launches (measurement builds, part_body.h)
        unsigned long long h[8];
        HIPCHK(hipMemcpyAsync(h, e->d_pprof.p, 8 * 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        const double w = h[5] ? (double)h[5] : 1.0;
        fprintf(stderr, "[part prof] kind %d waves %llu events/wave %.1f cycles/wave: setup %.0f stage %.0f loop %.0f end %.0f\n",
                ps.kind, h[5], h[4] / w, h[0] / w, h[1] / w, h[2] / w, h[3] / w);
      }
      ps.ran = true;
      any = true;
      bytes += (double)n * ev_bytes * ps.n_groups;
    }
    // K_slab: item = (key segment, group whose shape reads this stream)
    for (size_t si = 0; si < e->ssets.size(); ++si) {
      auto& ss = *e->ssets[si];
      if (ss.partition != pi) continue;
      const auto& gl = ss.glist[stream];
      if (gl.empty() || hv[1] == 0) continue;
      slab_grow_keys(e, ss, hv[0]);
      const int64_t items = (int64_t)hv[1] * (int64_t)gl.size();
      if (items > INT32_MAX) throw Error(SDH_E_UNSUPPORTED, "K_slab launch beyond 2^31 work items (split the batch)");
      ss.journal.ensure((size_t)items);
      ss.journal_idx.ensure((size_t)items);
      HIPCHK(hipMemsetAsync(ss.journal_idx.p, 0xff, (size_t)items * 8, e->stream));
      HIPCHK(hipMemcpyAsync(ss.head_bak.p, ss.head.p, ss.nsub * 8, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(hipMemcpyAsync(ss.live_bak.p, ss.live.p, 256 * 8, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(hipMemsetAsync(ss.traffic.p, 0, 256 * 8, e->stream));
      sdh::SlabLaunch S{};
      S.xcd = e->xcd;
      S.lconst = e->d_lconst.p;
      S.lc_slots = e->lc_slots;
      S.queries = e->d_gq.p;
      S.lane_q = e->d_lane_q.p;
      S.group_tmpl = e->d_group_tmpl.p;
      S.shapes = ss.d_shapes.p;
      S.group_shape = ss.d_group_shape.p;
      S.b = B;
      S.seg_begin = e->r_off.p;
      S.seg_len = e->r_cnt.p;
      S.seg_kid = e->r_uniq.p;
      S.key_of_id = rt.key_of_id.p;
      S.ev_idx = e->r_idx_s.p;
      S.glist = ss.d_glist[stream].p;
      S.n_glist = (int32_t)gl.size();
      S.n_items = (int32_t)items;
      S.groups = ss.n_groups;
      S.group_base = ss.group_base;
      S.dir = ss.dir.p;
      S.journal = ss.journal.p;
      S.journal_idx = ss.journal_idx.p;
      S.ring = ss.d_ring.p;
      S.ring_cap = ss.d_cap.p;
      S.head = ss.head.p;
      S.tail = ss.tail.p;
      S.nsub = ss.nsub;
      S.lds_words = ss.lds_words;
      S.max_na = 1;
      for (int g = 0; g < ss.n_groups; ++g)
        for (int st = 0; st < kg::GMAXSTREAM; ++st)
          S.max_na = std::max<int32_t>(S.max_na, e->gq[e->group_tmpl[ss.group_base + g]].n_cap[st]);
      S.live = ss.live.p;
      S.traffic = ss.traffic.p;
      S.out = e->g_out.p;
      S.out_cap = e->g_out_cap;
      S.out_next = e->g_out_next.p;
      S.rec_count = e->g_nrec.p;
      S.rec_off = e->g_rec_off.p;
      S.rec_cap = e->g_out_cap / NREC_MIN_WORDS + 1;
      S.rec_next = e->g_rec_next.p;
      S.write_records = write ? 1 : 2;
      S.err = e->d_serr.p + 4 * si;
      // two LDS tiers: every item first with small rows (more resident waves); the few whose block
      // outgrows them are deferred to a second launch with the set's full rows
      const int small = std::min(ss.lds_words, e->slab_lds_small);
      if (small < ss.lds_words) {
        ss.defer.ensure((size_t)items);
        ss.defer_n.ensure(1);
        HIPCHK(hipMemsetAsync(ss.defer_n.p, 0, 4, e->stream));
        S.lds_words = small;
        S.defer_cap = (int32_t)items;
        S.defer = ss.defer.p;
        S.defer_n = ss.defer_n.p;
      }
      HIPCHK(sdh_launch_slab(&S, e->stream));
      if (small < ss.lds_words) {
        int32_t nd = 0;
        d2h_sync(e, &nd, ss.defer_n.p, 4);
        if (nd > 0) {
          sdh::SlabLaunch D = S;
          D.lds_words = ss.lds_words;
          D.defer_cap = 0;
          D.item_list = ss.defer.p;
          D.n_items = std::min<int32_t>(nd, (int32_t)items);
          HIPCHK(sdh_launch_slab(&D, e->stream));
        }
        ss.deferred += nd;
      }
      ss.items = items;
      e->slab_items += items;
      any = true;
      // every item reads its directory word and its key's events; the block bytes it moves are
      // counted by the kernel (added once the pass has run)
      bytes += (double)n * ev_bytes * gl.size() + (double)items * 8;
    }
  }
  *bytes_out = bytes;
  return any;
}

// one K_gen step for every set fed by `stream`
void launch_gen(sdh_engine* e, int stream, const StreamBatch& B, double* ms_out, double* bytes_out) {
  *ms_out = 0;
  *bytes_out = 0;
  e->stats.last_gen_items = 0;
  e->stats.last_seq_items = 0;
  if (e->gsets.empty() && e->psets.empty() && e->ssets.empty()) return;
  const int64_t n = B.n;
  e->g_out_cap = std::max<int64_t>(e->g_out_cap, std::max<int64_t>(1 << 22, n * 64));
  static_assert((1 << 22) > 2 * GEN_RING_MARGIN, "ring capacity");
  e->d_err.ensure(4);
  e->g_rec_next.ensure(1);
  const bool write = (e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) == 0;
  // the blocks a pass modifies are journaled so that an overflow (match output, K_part tables, K_gen
  // pools, K_slab space) can be undone and the push re-run exactly at the grown capacity, in both
  // output modes (device records grow like the match table's records: no push drops a match)
  e->g_journal = true;
  for (auto& up : e->gsets) up->jn = 0;
  for (auto& ss : e->ssets) slab_prepare(e, *ss);
  const size_t nss = e->ssets.size();
  std::vector<int32_t> serr(4 * std::max<size_t>(1, nss), 0);
  double bytes = 0;
  int32_t tail_len = -1;
  bool any = false;
  int32_t errs[4] = {0, 0, 0, 0};
  unsigned long long nrec = 0, used = 0;
  float ms = 0;
  const size_t nps = e->psets.size();
  std::vector<int32_t> perr(4 * std::max<size_t>(1, nps), 0);
  for (int attempt = 0;; ++attempt) {
    e->g_out.ensure((size_t)e->g_out_cap);
    if (write) e->g_rec_off.ensure((size_t)(e->g_out_cap / NREC_MIN_WORDS + 1));  // a record has at least NREC_MIN_WORDS words (the narrow ones)
    HIPCHK(hipMemsetAsync(e->d_err.p, 0, 16, e->stream));
    HIPCHK(hipMemsetAsync(e->d_perr.p, 0, perr.size() * 4, e->stream));
    HIPCHK(hipMemsetAsync(e->d_serr.p, 0, serr.size() * 4, e->stream));
    e->slab_items = 0;
    HIPCHK(hipMemsetAsync(e->g_out_next.p, 0, 8, e->stream));
    HIPCHK(hipMemsetAsync(e->g_nrec.p, 0, 8, e->stream));
    HIPCHK(hipMemsetAsync(e->g_rec_next.p, 0, 8, e->stream));
    HIPCHK(hipEventRecord(e->ev0, e->stream));
    any = gen_pass(e, stream, B, write, &bytes, &tail_len);
    HIPCHK(hipEventRecord(e->ev1, e->stream));
    HIPCHK(hipMemcpyAsync(errs, e->d_err.p, 16, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(perr.data(), e->d_perr.p, perr.size() * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(serr.data(), e->d_serr.p, serr.size() * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&nrec, e->g_nrec.p, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&used, e->g_out_next.p, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipEventElapsedTime(&ms, e->ev0, e->ev1));
    bool out_over = errs[2] != 0, part_over = false, slab_over = false;
    for (size_t i = 0; i < nps; ++i) {
      out_over |= perr[4 * i + 2] != 0;
      part_over |= perr[4 * i] != 0;
    }
    for (size_t i = 0; i < nss; ++i) {
      out_over |= serr[4 * i + 2] != 0;
      slab_over |= serr[4 * i] != 0 || serr[4 * i + 1] != 0;
    }
    kg::Sizing grown;
    const bool pools_over = errs[0] != 0 && gen_grown_sizing(e, errs[0], &grown);
    if (sdh::knob("SDH_TRACE"))
      fprintf(stderr, "[sdh] gen pass stream %d n %lld attempt %d: out %d part %d pools %d slab %d, %llu of %lld words, %.2f ms\n",
              stream, (long long)n, attempt, (int)out_over, (int)part_over, (int)pools_over, (int)slab_over, used,
              (long long)e->g_out_cap, ms);
    if ((out_over || part_over || pools_over || slab_over) && e->g_journal && attempt < 24 &&
        (!errs[0] || pools_over) && !errs[1] && !errs[3]) {
      // undo the pass (K_gen blocks from the journal; K_part tables are double-buffered and their
      // per-key selectors are swapped only after success) and re-run it with room for every match
      // record (out_next counts the words every record asked for), every K_part partial and the
      // K_gen pools / lists that overflowed
      gen_restore_journal(e);
      for (size_t i = 0; i < nss; ++i) {
        auto& ss = *e->ssets[i];
        std::vector<int64_t> demand(ss.nsub, 0);
        if (serr[4 * i + 1] && ss.items > 0) {  // what the push tried to take from each ring
          std::vector<unsigned long long> h(ss.nsub);
          HIPCHK(hipMemcpy(h.data(), ss.head.p, ss.nsub * 8, hipMemcpyDeviceToHost));
          for (int r = 0; r < ss.nsub; ++r) demand[r] = (int64_t)(h[r] - ss.h_push0[r]);
        }
        slab_rollback(e, ss);
        if (serr[4 * i]) {  // a block outgrew the LDS staging area
          if (ss.lds_words >= 13312) throw Error(SDH_E_CAPACITY, "K_slab: more partials in one (key, group) block "
                                                                 "than the LDS staging area holds");
          ss.lds_words = std::min(13312, 2 * ss.lds_words);
        }
        if (serr[4 * i + 1]) slab_prepare(e, ss, &demand);  // a ring ran out of room: reclaim / grow
      }
      if (pools_over) {
        gen_relayout(e, grown, true);  // (the next pass journals its blocks in the new layout)
        ++e->gen_regrows;
      }
      if (out_over)
        while (e->g_out_cap < (int64_t)used + (int64_t)used / 4 + GEN_RING_MARGIN) e->g_out_cap *= 2;
      for (size_t i = 0; i < nps; ++i)
        if (perr[4 * i]) {
          if (e->psets[i]->cap >= (1 << 16))
            throw Error(SDH_E_CAPACITY, "more than 65536 pending partials in one K_part instance");
          part_grow_cap(e, *e->psets[i]);
        }
      continue;
    }
    if (part_over)
      throw Error(SDH_E_CAPACITY, "K_part partial table overflow (no room for an exact re-run)");
    if (out_over)
      throw Error(SDH_E_CAPACITY, "K_gen match output overflow (no room for an exact re-run)");
    if (slab_over) throw Error(SDH_E_CAPACITY, "K_slab capacity (no room for an exact re-run)");
    break;
  }
  // the push succeeded: its K_slab allocations are committed (the heads tell the next push's room)
  for (auto& up : e->ssets) {
    auto& ss = *up;
    if (ss.items <= 0) continue;
    slab_heads(e, ss);
    unsigned long long tr[256];
    HIPCHK(hipMemcpy(tr, ss.traffic.p, sizeof tr, hipMemcpyDeviceToHost));
    for (unsigned long long x : tr) bytes += (double)x;
    ss.items = 0;
  }
  // the push succeeded: the K_part tables it wrote become current
  for (auto& pp : e->psets)
    if (pp->ran) {
      std::swap(pp->cur.p, pp->nxt.p);
      std::swap(pp->cur.n, pp->nxt.n);
      pp->ran = false;
    }
  if (tail_len >= 0 && !errs[0] && !errs[1] && !errs[3]) {
    HIPCHK(sdh_seq_tail(&B, e->seq_tail[stream].p, e->seq_tail_len[stream], tail_len, e->stream));
    e->seq_tail_len[stream] = tail_len;
  }
  *ms_out = ms;
  *bytes_out = bytes;
  if (errs[3]) throw Error(SDH_E_CAPACITY, "partition key table full");
  if (errs[1]) throw Error(SDH_E_REFERENCE, "the reference engine would throw on this stream "
                                            "(ConcurrentModification / IllegalState / NullPointer)");
  if (errs[0]) throw Error(SDH_E_CAPACITY, (errs[0] & kg::CAP_FIXED)
                                               ? "K_gen compiled-in limit exceeded (GC pin depth)"
                                               : "K_gen instance pools could not grow further (4096 StateEvents / nodes per "
                                                 "instance, or device memory)");
  if (!any) nrec = used = 0;
  *bytes_out += (double)nrec * 32.0;  // one (query, ts, seqs) record per match, as for K_ratchet
  e->stats.matches += (int64_t)nrec;
  e->g_dev_matches = (int64_t)nrec;
  e->g_used = (int64_t)used;
}

// Host-resident batch -> HBM (the StreamJunction -> receiver hand-off of north_star (2)): the
// columns go to one device buffer over the side stream `h2d`; pinned caller memory is copied
// directly, pageable memory through two pinned staging slots whose host copy of slice i+1 overlaps
// the DMA of slice i. The compute stream waits on the transfer's event.
void stage_host_batch(sdh_engine* e, const sdh_batch* b, StreamBatch& B) {
  const int na = B.n_attr;
  const int64_t n = b->n;
  struct Part {
    const void* src;
    size_t bytes, off;
  };
  std::vector<Part> parts;
  size_t total = 0;
  auto add = [&](const void* src, size_t bytes) {
    total = (total + 255) & ~(size_t)255;
    parts.push_back({src, bytes, total});
    total += bytes;
  };
  add(b->ts, (size_t)n * 8);
  for (int a = 0; a < na; ++a) add(b->cols[a], (size_t)n * B.width[a]);
  for (int a = 0; a < na; ++a)
    if (b->nulls && b->nulls[a]) add(b->nulls[a], (size_t)n);
  e->d_batch.ensure(total);
  float ms = 0;
  HIPCHK(hipEventRecord(e->ev_h0, e->h2d));
  const size_t SLICE = (size_t)4 << 20;
  for (const Part& p : parts) {
    hipPointerAttribute_t at{};
    const bool pinned = hipPointerGetAttributes(&at, p.src) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    uint8_t* dst = e->d_batch.p + p.off;
    if (pinned) {
      HIPCHK(hipMemcpyAsync(dst, p.src, p.bytes, hipMemcpyHostToDevice, e->h2d));
      continue;
    }
    for (size_t o = 0; o < p.bytes; o += SLICE) {
      const size_t len = std::min(SLICE, p.bytes - o);
      const int slot = e->stage_next;
      e->stage_next ^= 1;
      e->stage[slot].ensure(SLICE);
      HIPCHK(hipEventSynchronize(e->ev_stage[slot]));  // the slot's previous DMA has drained
      memcpy(e->stage[slot].p, (const uint8_t*)p.src + o, len);
      HIPCHK(hipMemcpyAsync(dst + o, e->stage[slot].p, len, hipMemcpyHostToDevice, e->h2d));
      HIPCHK(hipEventRecord(e->ev_stage[slot], e->h2d));
    }
  }
  HIPCHK(hipEventRecord(e->ev_h1, e->h2d));
  HIPCHK(hipStreamWaitEvent(e->stream, e->ev_h1, 0));
  HIPCHK(hipEventSynchronize(e->ev_h1));
  HIPCHK(hipEventElapsedTime(&ms, e->ev_h0, e->ev_h1));
  e->stats.last_ingest_ms = ms;
  e->stats.ingest_bytes += (int64_t)total;
  size_t k = 0;
  B.ts = (const int64_t*)(e->d_batch.p + parts[k++].off);
  for (int a = 0; a < na; ++a) B.col[a] = e->d_batch.p + parts[k++].off;
  for (int a = 0; a < na; ++a) {
    B.nul[a] = nullptr;
    if (b->nulls && b->nulls[a]) B.nul[a] = e->d_batch.p + parts[k++].off;
  }
}

int do_push(sdh_engine* e, int32_t stream, const sdh_batch* b) {
  if (!b || stream < 0 || stream >= (int)e->prog.stream_types.size())
    throw Error(SDH_E_INVALID, "bad stream or batch");
  const auto& types = e->prog.stream_types[stream];
  const int na = (int)types.size();
  if (b->n_cols != na) throw Error(SDH_E_INVALID, fmt("stream %d has %d attributes, batch has %d", stream, na, b->n_cols));
  if (b->n < 0 || (e->cfg.max_batch > 0 && b->n > e->cfg.max_batch))
    throw Error(SDH_E_INVALID, "batch larger than max_batch");
  if (b->n == 0) return SDH_OK;
  check_fan_strings(e, stream);
  HIPCHK(hipSetDevice(e->dev));
  // an exact re-run needs the journal of the K_gen blocks the push modifies (gen_journal): a batch
  // whose bound does not fit a third of free HBM is pushed as two halves -- the same events in the
  // same order, so the same matches
  if (!e->gsets.empty() && b->n > 1) {
    size_t fr = 0, tot = 0;
    const char* jb = sdh::knob("SDH_JOURNAL_BUDGET");  // (tests: force the split)
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && gen_journal_bound(e, b->n) > (jb ? atof(jb) : (double)fr / 3)) {
      std::vector<const void*> c0(na), c1(na);
      std::vector<const uint8_t*> n0(na), n1(na);
      const int64_t h = b->n / 2;
      for (int a = 0; a < na; ++a) {
        c0[a] = b->cols[a];
        c1[a] = (const uint8_t*)b->cols[a] + h * attr_width(types[a]);
        n0[a] = b->nulls ? b->nulls[a] : nullptr;
        n1[a] = (b->nulls && b->nulls[a]) ? b->nulls[a] + h : nullptr;
      }
      sdh_batch first = *b, second = *b;
      first.n = h;
      first.cols = c0.data();
      first.nulls = b->nulls ? n0.data() : nullptr;
      second.n = b->n - h;
      second.ts = b->ts + h;
      second.cols = c1.data();
      second.nulls = b->nulls ? n1.data() : nullptr;
      do_push(e, stream, &first);
      return do_push(e, stream, &second);
    }
  }
  (void)hipGetLastError();
  StreamBatch B{};
  B.n = b->n;
  B.n_attr = na;
  B.stream = stream;
  B.seq_base = e->seq;
  B.prev_ts = e->prev_ts[stream];
  for (int a = 0; a < na; ++a) B.width[a] = attr_width(types[a]);
  if (b->on_device) {
    B.ts = b->ts;
    for (int a = 0; a < na; ++a) {
      B.col[a] = b->cols[a];
      B.nul[a] = b->nulls ? b->nulls[a] : nullptr;
    }
  } else {
    stage_host_batch(e, b, B);
  }
  std::vector<int> qs;
  for (int li = 0; li < (int)e->lq.size(); ++li)
    if (std::find(e->lq[li].streams.begin(), e->lq[li].streams.end(), stream) != e->lq[li].streams.end())
      qs.push_back(li);
  int64_t t01[2];
  if (b->on_device) {
    d2h_sync(e, &t01[0], B.ts, 8);
    d2h_sync(e, &t01[1], B.ts + (b->n - 1), 8);
  } else {
    t01[0] = b->ts[0];
    t01[1] = b->ts[b->n - 1];
  }
  double ms = 0, bytes = 0;
  int64_t consumers = 0;
  if (!e->started) {  // the runtime starts with its first event unless sdh_engine_start said when
    e->started = true;
    e->start_ts = t01[0];
  }
  // the previous push's device-only matches (SDH_FLAG_DEVICE_MATCHES) are dropped here
  e->work.clear();
  e->device_matches = 0;
  e->r_blocks_used = 0;
  e->r_blk_taken = 0;
  e->r_matches = 0;
  e->g_dev_matches = 0;
  e->g_used = 0;
  e->dev_polled = false;
  e->last_n = b->n;
  e->last_seq_base = B.seq_base;
  for (auto& k : e->part_kept) k = b->n;
  try {
    if (!qs.empty()) {
      bool unordered = false;
      launch(e, stream, B, t01, qs, true, &unordered);
      bool chunked = false;
      for (auto& w : e->work) chunked |= w.n_chunks > 1;
      if (unordered && chunked) launch(e, stream, B, t01, qs, false, &unordered);  // exact fallback
      for (int li : qs) e->cur[li] ^= 1;
      ms += e->stats.last_kernel_ms;
      bytes += e->stats.last_kernel_bytes;
      consumers += (int64_t)qs.size();
    }
    // K_gen before K_ratchet: a push whose only matches are K_ratchet's places them directly
    double gms = 0, gbytes = 0;
    e->stats.last_gen_items = 0;
    e->stats.last_seq_items = 0;
    launch_gen(e, stream, B, &gms, &gbytes);
    ms += gms;
    bytes += gbytes;
    launch_ratchet(e, stream, B, t01);
    for (const auto& g : e->rg)
      if (g.stream == stream) consumers += g.n_lanes;
    ms += e->r_kernel_ms;
    bytes += e->r_kernel_bytes;
  } catch (const std::exception& ex) {
    // kernels may already have advanced part of the state: the engine no longer mirrors the
    // reference, so every later call fails (restore a snapshot or recreate)
    e->prev_ts[stream] = t01[1];
    e->seq += b->n;
    e->broken = ex.what();
    throw;
  }
  // (event, query) evaluations: a partition's queries see only the events routed to a key of this
  // engine (null keys and other ranks' keys are not evaluated)
  int64_t pe = b->n * consumers;
  for (const auto& g : e->gq)
    if (g.recv_n[stream] > 0) {
      ++consumers;
      pe += g.partition >= 0 && g.partition < (int)e->part_kept.size() ? e->part_kept[g.partition] : b->n;
    }
  if (consumers) {
    e->stats.pattern_events += pe;
    e->stats.matches += e->device_matches + e->r_matches;
    e->stats.last_kernel_ms = ms;
    e->stats.last_kernel_bytes = bytes;
  }
  e->prev_ts[stream] = t01[1];
  e->seq += b->n;
  e->stats.events += b->n;
  // the push is committed; its matches join the device table (R18-sorted at poll), or, when they
  // all come from K_ratchet, are already at their R18 rows (placed by the launch: no sort at poll)
  if (!(e->cfg.flags & SDH_FLAG_DEVICE_MATCHES)) {
    const bool only_ratchet = e->device_matches == 0 && e->g_dev_matches == 0;
    if (e->r_placing) {
      place_commit(e, B.ts, B.seq_base, b->n);
    } else if (!(only_ratchet && e->r_matches == 0)) {
      placed_to_table(e);
      const int64_t n0 = e->mt.n;
      append_chain(e);
      append_ratchet(e, B.ts, B.seq_base);
      append_gen(e, B.ts, B.seq_base, stream);
      if (e->ck.active) chunk_rows(e, n0);
    }
  }
  return SDH_OK;
}

// knobs.h: the knobs of the engine whose ABI call runs on this thread
thread_local const std::vector<std::pair<std::string, std::string>>* t_knobs = nullptr;
struct KnobScope {
  const std::vector<std::pair<std::string, std::string>>* prev;
  explicit KnobScope(const sdh_engine* e) : prev(t_knobs) { t_knobs = e ? &e->knobs : nullptr; }
  ~KnobScope() { t_knobs = prev; }
};

template <class F>
int guard(sdh_engine* e, F f) {
  KnobScope ks(e);
  try {
    return f();
  } catch (const Error& ex) {
    if (e) e->err = ex.what();
    return ex.code;
  } catch (const std::exception& ex) {
    if (e) e->err = ex.what();
    return SDH_E_INVALID;
  }
}

void check_usable(sdh_engine* e) {
  if (!e->broken.empty())
    throw Error(SDH_E_CAPACITY, "engine state is undefined after a failed push (" + e->broken +
                                    "); restore a snapshot or create a new engine");
}

// R18-sorted matches since the last poll; host == false leaves them in HBM (sdh_engine_poll_device)
// The window's matches R18-sorted into the ABI arrays in HBM (po_*; *tw words); with `kw_spec`
// (chunk words, lo words: sdh_engine_gather) also each row's merge key into x_keys.
int64_t poll_sorted(sdh_engine* e, int64_t* tw, const int* kw_spec = nullptr) {
  int64_t n = 0;
  *tw = 0;
  const int kw = kw_spec ? 2 * kw_spec[0] + 1 + 3 * kw_spec[1] : 0;
  if (kw) e->x_keys.ensure((size_t)std::max<int64_t>(1, e->mt.n) * kw);
  if (e->mt.placed) {  // compact rows already in R18 order (place_ratchet): 4 words per match
    n = e->mt.n;
    *tw = 4 * n;
    poll_reserve(e, n, *tw);
    HIPCHK(sdh_compact_fill(e->pc_rows.p, e->cw, n, e->ts_log.p, e->seq_ref, e->po_q.p, e->po_key.p, e->po_ts.p,
                            e->po_seq.p, e->po_tb.p, e->po_off.p, e->po_words.p, e->stream));
    if (kw)
      HIPCHK(sdh_merge_keys_placed(e->pc_rows.p, e->cw, n, e->seq_ref, e->d_out_rank.p, e->d_qinfo.p,
                                   (int)e->prog.stream_types.size(), kw_spec[0], kw_spec[1], e->x_keys.p, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  } else if (e->mt.n > 0) {
    n = e->mt.n;
    const int32_t* perm = table_order(e, tw);
    e->po_words.ensure((size_t)std::max<int64_t>(*tw, 1));
    HIPCHK(sdh_poll_words(table_view(e), perm, n, e->po_off.p, e->po_words.p, e->stream));
    if (kw)
      HIPCHK(sdh_merge_keys_table(table_view(e), perm, n, kw_spec[0], kw_spec[1], e->mt.chunked ? 1 : 0, e->x_keys.p,
                                  e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  if (n == 0) {
    e->po_off.ensure(1);
    HIPCHK(hipMemsetAsync(e->po_off.p, 0, 8, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return n;
}

int do_poll(sdh_engine* e, sdh_matches* out, bool host) {
  check_usable(e);
  int64_t tw = 0;
  const int64_t n = poll_sorted(e, &tw);
  if (host) {  // (pinned; sized like poll_reserve's device arrays)
    const int64_t hn = std::max<int64_t>(n, POLL_MIN_ROWS);
    e->ho_q.ensure(hn);
    e->ho_key.ensure(hn);
    e->ho_ts.ensure(hn);
    e->ho_seq.ensure(hn);
    e->ho_tb.ensure(hn);
    e->ho_off.ensure(hn + 1);
    e->ho_words.ensure(std::max<int64_t>(tw, 4 * POLL_MIN_ROWS));
    e->ho_off.p[0] = 0;
    if (n) {
      HIPCHK(hipMemcpyAsync(e->ho_q.p, e->po_q.p, n * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipMemcpyAsync(e->ho_key.p, e->po_key.p, n * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipMemcpyAsync(e->ho_ts.p, e->po_ts.p, n * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipMemcpyAsync(e->ho_seq.p, e->po_seq.p, n * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipMemcpyAsync(e->ho_tb.p, e->po_tb.p, n * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipMemcpyAsync(e->ho_off.p, e->po_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, e->stream));
      if (tw) HIPCHK(hipMemcpyAsync(e->ho_words.p, e->po_words.p, tw * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
    }
    out->query = e->ho_q.p;
    out->key = e->ho_key.p;
    out->ts = e->ho_ts.p;
    out->seq = e->ho_seq.p;
    out->tb = e->ho_tb.p;
    out->off = e->ho_off.p;
    out->words = e->ho_words.p;
  } else {
    out->query = e->po_q.p;
    out->key = e->po_key.p;
    out->ts = e->po_ts.p;
    out->seq = e->po_seq.p;
    out->tb = e->po_tb.p;
    out->off = e->po_off.p;
    out->words = e->po_words.p;
  }
  out->n = n;
  table_clear(e);
  return SDH_OK;
}

// the window's matches as compact rows (sdh_engine_poll_compact): a placed window hands out its rows
// as they are; otherwise the table is R18-sorted and converted, and a row the form cannot express
// fails the call with the window left pending
int do_poll_compact(sdh_engine* e, sdh_matches_compact* out, bool device) {
  check_usable(e);
  const int64_t n = e->mt.n;
  const int w = e->cw;
  if (!e->mt.placed && n) {
    if (e->seq - e->seq_ref >= INT32_MAX) throw Error(SDH_E_UNSUPPORTED, "compact rows: seq span past 2^31");
    int64_t tw = 0;
    const int32_t* perm = table_order(e, &tw);
    e->pc_rows.ensure((size_t)(n * w));
    e->pc_err.ensure(1);
    HIPCHK(hipMemsetAsync(e->pc_err.p, 0, 4, e->stream));
    HIPCHK(sdh_table_compact(table_view(e), perm, n, w, e->seq_ref, e->pc_rows.p, e->pc_err.p, e->stream));
    int32_t bad = 0;
    d2h_sync(e, &bad, e->pc_err.p, 4);
    if (bad)
      throw Error(SDH_E_UNSUPPORTED, "compact rows: a match has a count-state chain, a partition key or a timer "
                                     "(poll it with sdh_engine_poll)");
  }
  e->pc_rows.ensure(1);
  out->n = n;
  out->seq_base = e->seq_ref;
  out->width = w;
  out->flags = 0;
  if (device) {
    out->rows = e->pc_rows.p;
  } else {
    e->hc_rows.ensure((size_t)std::max<int64_t>(n * w, POLL_MIN_ROWS * w));
    if (n) d2h_sync(e, e->hc_rows.p, e->pc_rows.p, (size_t)(n * w) * 4);
    out->rows = e->hc_rows.p;
  }
  table_clear(e);
  return SDH_OK;
}

// sdh_engine_poll_compact_ex: every match as a compact row, chains in a side array, keys and timer
// tiebreaks beside the rows
int do_poll_compact_ex(sdh_engine* e, sdh_matches_compact_ex* out, bool device) {
  check_usable(e);
  const int64_t n = e->mt.n;
  const int w = e->cw;
  const bool want_key = !e->lp.parts.empty(), want_tb = e->has_absent;
  int64_t nch = 0;
  const size_t rows = (size_t)std::max<int64_t>(1, n);
  if (want_key) e->px_key.ensure(rows);
  if (want_tb) e->px_tb.ensure(rows);
  e->px_chain.ensure(1);
  if (!e->mt.placed && n) {
    if (e->seq - e->seq_ref >= INT32_MAX) throw Error(SDH_E_UNSUPPORTED, "compact rows: seq span past 2^31");
    int64_t tw = 0;
    const int32_t* perm = table_order(e, &tw);
    e->px_cw.ensure((size_t)n + 1);
    e->px_temp.ensure(sdh_ex_temp_bytes(n));
    HIPCHK(sdh_ex_chain_words(table_view(e), perm, n, e->px_cw.p, e->px_temp.p, e->px_temp.n, e->stream));
    HIPCHK(hipMemcpyAsync(&nch, e->px_cw.p + n, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->pc_rows.ensure((size_t)(n * w));
    e->px_chain.ensure((size_t)std::max<int64_t>(1, nch));
    e->pc_err.ensure(1);
    HIPCHK(hipMemsetAsync(e->pc_err.p, 0, 4, e->stream));
    HIPCHK(sdh_ex_rows(table_view(e), perm, n, w, e->seq_ref, e->px_cw.p, e->pc_rows.p, e->px_chain.p,
                       want_key ? e->px_key.p : nullptr, want_tb ? e->px_tb.p : nullptr, e->pc_err.p, e->stream));
    int32_t bad = 0;
    d2h_sync(e, &bad, e->pc_err.p, 4);
    if (bad) throw Error(SDH_E_UNSUPPORTED, "compact rows: a seq distance past 2^31 (poll it with sdh_engine_poll)");
  } else if (n) {  // placed K_ratchet rows: no key, no timer
    if (want_key) HIPCHK(sdh_fill_i64(e->px_key.p, n, -1, e->stream));
    if (want_tb) HIPCHK(sdh_fill_i64(e->px_tb.p, n, INT64_MIN, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  e->pc_rows.ensure(1);
  out->n = n;
  out->seq_base = e->seq_ref;
  out->width = w;
  out->flags = 0;
  out->n_chain = nch;
  if (device) {
    out->rows = e->pc_rows.p;
    out->key = want_key ? e->px_key.p : nullptr;
    out->tb = want_tb ? e->px_tb.p : nullptr;
    out->chain = e->px_chain.p;
  } else {
    e->hc_rows.ensure((size_t)std::max<int64_t>(n * w, POLL_MIN_ROWS * w));
    e->hx_chain.ensure((size_t)std::max<int64_t>(nch, 1));
    if (n) HIPCHK(hipMemcpyAsync(e->hc_rows.p, e->pc_rows.p, (size_t)(n * w) * 4, hipMemcpyDeviceToHost, e->stream));
    if (nch) HIPCHK(hipMemcpyAsync(e->hx_chain.p, e->px_chain.p, (size_t)nch * 4, hipMemcpyDeviceToHost, e->stream));
    if (want_key) {
      e->hx_key.ensure(rows);
      if (n) HIPCHK(hipMemcpyAsync(e->hx_key.p, e->px_key.p, (size_t)n * 8, hipMemcpyDeviceToHost, e->stream));
    }
    if (want_tb) {
      e->hx_tb.ensure(rows);
      if (n) HIPCHK(hipMemcpyAsync(e->hx_tb.p, e->px_tb.p, (size_t)n * 8, hipMemcpyDeviceToHost, e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    out->rows = e->hc_rows.p;
    out->key = want_key ? e->hx_key.p : nullptr;
    out->tb = want_tb ? e->hx_tb.p : nullptr;
    out->chain = e->hx_chain.p;
  }
  table_clear(e);
  return SDH_OK;
}

// ---- multi-GPU exchange (comm.h) ----
template <class F>
void xcall(F f) {
  try {
    f();
  } catch (const Error&) {
    throw;
  } catch (const std::invalid_argument& ex) {
    throw Error(SDH_E_INVALID, ex.what());
  } catch (const std::runtime_error& ex) {
    throw Error(SDH_E_DEVICE, ex.what());
  }
}

int push_chunk(sdh_engine* e, int32_t stream, const sdh_batch* b);

// sdh_engine_push_bcast: the root's batch (staged into HBM first when it is host-resident) goes to
// every rank -- a header {n, stream, chunk, null-mask bits}, then ts, the attribute columns and the
// null masks the header names -- and every rank pushes it from HBM.
int do_push_bcast(sdh_engine* e, int32_t stream, const sdh_batch* b, int root) {
  if (!e->comm) throw Error(SDH_E_INVALID, "sdh_engine_push_bcast: no communicator (sdh_engine_set_comm)");
  HIPCHK(hipSetDevice(e->dev));
  const bool am_root = xch::rank(e->comm) == root;
  int64_t hdr[xch::HDR] = {};
  StreamBatch B{};
  if (am_root && (!b || stream < 0 || stream >= (int)e->prog.stream_types.size() ||
                  b->n_cols != (int)e->prog.stream_types[stream].size() || b->n < 0)) {
    // an invalid batch still takes part in the collective, as an error header: every rank then fails
    // this call with SDH_E_INVALID (no rank waits on a broadcast the root never makes)
    hdr[0] = -1;
    xcall([&] { xch::bcast_hdr(e->comm, hdr, root, e->stream); });
    throw Error(SDH_E_INVALID, "bad stream or batch");
  }
  if (am_root) {
    const int na = b->n_cols;
    B.n = b->n;
    B.n_attr = na;
    for (int a = 0; a < na; ++a) B.width[a] = attr_width(e->prog.stream_types[stream][a]);
    if (b->n > 0 && !b->on_device) {
      stage_host_batch(e, b, B);
    } else {
      B.ts = b->ts;
      for (int a = 0; a < na; ++a) {
        B.col[a] = b->cols[a];
        B.nul[a] = b->nulls ? b->nulls[a] : nullptr;
      }
    }
    int64_t mask = 0;
    for (int a = 0; a < na; ++a)
      if (B.nul[a]) mask |= (int64_t)1 << a;
    hdr[0] = b->n;
    hdr[1] = stream;
    hdr[2] = b->chunk;
    hdr[3] = mask;
  }
  xcall([&] { xch::bcast_hdr(e->comm, hdr, root, e->stream); });
  const int64_t n = hdr[0];
  if (n < 0) throw Error(SDH_E_INVALID, "sdh_engine_push_bcast: the root's batch was invalid (bad stream or batch)");
  stream = (int32_t)hdr[1];
  if (stream < 0 || stream >= (int)e->prog.stream_types.size()) throw Error(SDH_E_INVALID, "broadcast: bad stream");
  const auto& types = e->prog.stream_types[stream];
  const int na = (int)types.size();
  if (n == 0) return SDH_OK;
  // the receivers' layout (256-B aligned parts in x_batch), the root's sources
  std::vector<xch::Buf> bufs;
  size_t total = 0;
  auto add = [&](const void* src, size_t bytes) {
    total = (total + 255) & ~(size_t)255;
    bufs.push_back({src, (void*)(uintptr_t)total, bytes});
    total += bytes;
  };
  add(B.ts, (size_t)n * 8);
  for (int a = 0; a < na; ++a) add(am_root ? B.col[a] : nullptr, (size_t)n * attr_width(types[a]));
  for (int a = 0; a < na; ++a)
    if (hdr[3] >> a & 1) add(am_root ? B.nul[a] : nullptr, (size_t)n);
  if (!am_root) {
    e->x_batch.ensure(total);
    for (auto& x : bufs) x.dst = e->x_batch.p + (uintptr_t)x.dst;
  }
  xcall([&] { xch::bcast_bufs(e->comm, bufs, root, e->stream); });
  std::vector<const void*> cols((size_t)na);
  std::vector<const uint8_t*> nuls((size_t)na, nullptr);
  auto at = [&](size_t i) -> const void* { return am_root ? bufs[i].src : bufs[i].dst; };
  size_t k = 1;
  for (int a = 0; a < na; ++a) cols[(size_t)a] = at(k++);
  for (int a = 0; a < na; ++a)
    if (hdr[3] >> a & 1) nuls[(size_t)a] = (const uint8_t*)at(k++);
  sdh_batch db{};
  db.n = n;
  db.ts = (const int64_t*)at(0);
  db.cols = cols.data();
  db.nulls = hdr[3] ? nuls.data() : nullptr;
  db.n_cols = na;
  db.on_device = 1;
  db.chunk = (int32_t)hdr[2];
  if (db.chunk && n > 1) return push_chunk(e, stream, &db);
  return do_push(e, stream, &db);
}

// sdh_engine_gather: this rank's sorted run and its merge keys go to rank 0 (a header {n, words,
// seq_ref, kw, seq} first), which merges the world's runs on the device (comm.hip sdh_merge_runs).
int do_gather(sdh_engine* e, sdh_matches* out, bool host) {
  if (!e->comm) throw Error(SDH_E_INVALID, "sdh_engine_gather: no communicator (sdh_engine_set_comm)");
  const int me = xch::rank(e->comm), W = xch::world(e->comm);
  if (e->cfg.shard_world != W || e->cfg.shard_rank != me)
    throw Error(SDH_E_INVALID, fmt("sdh_engine_gather: the engine is shard %d of %d, the communicator's rank %d of %d",
                                   e->cfg.shard_rank, e->cfg.shard_world, me, W));
  HIPCHK(hipSetDevice(e->dev));
  // the key words every rank uses (the same on all: same program, same pushes)
  const int spec[2] = {e->mt.chunk_pushed ? 1 : 0, e->has_absent ? 1 : 0};
  const int kw = 2 * spec[0] + 1 + 3 * spec[1];
  int64_t tw = 0;
  const int64_t n = poll_sorted(e, &tw, spec);
  int64_t hdr[xch::HDR] = {n, tw, e->seq_ref, kw, e->seq, 0, 0, 0};
  std::vector<int64_t> all((size_t)W * xch::HDR);
  xcall([&] { xch::gather_hdr(e->comm, hdr, all.data(), e->stream); });
  const bool local = xch::is_local(e->comm);
  // the poll windows must agree (same pushes since the last gather): with RCCL every rank holds every
  // header and refuses a mismatch before any rank clears its table or sends; the local
  // communicator's rank 0 checks before it clears its own
  for (int r = 0; r < W && (!local || me == 0); ++r) {
    const int64_t* h = all.data() + (size_t)r * xch::HDR;
    if (h[2] != hdr[2] || h[3] != kw || h[4] != hdr[4])
      throw Error(SDH_E_INVALID, fmt("sdh_engine_gather: rank %d's poll window differs from rank %d's (pushes out of step)", r, me));
  }
  const std::vector<xch::Buf> mine = {
      {e->po_q.p, nullptr, (size_t)n * 8},    {e->po_key.p, nullptr, (size_t)n * 8},
      {e->po_ts.p, nullptr, (size_t)n * 8},   {e->po_seq.p, nullptr, (size_t)n * 8},
      {e->po_tb.p, nullptr, (size_t)n * 8},   {e->po_off.p, nullptr, (size_t)(n + 1) * 8},
      {e->po_words.p, nullptr, (size_t)tw * 8}, {e->x_keys.p, nullptr, (size_t)n * kw * 8}};
  if (me != 0) {
    xcall([&] { xch::gather_bufs(e->comm, mine, {}, e->stream); });
    HIPCHK(hipStreamSynchronize(e->stream));  // (the sends drained before the buffers change)
    table_clear(e);
    poll_reserve(e, 0, 0);
    HIPCHK(hipMemsetAsync(e->po_off.p, 0, 8, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    *out = sdh_matches{0, e->po_q.p, e->po_key.p, e->po_ts.p, e->po_off.p, e->po_words.p, e->po_seq.p, e->po_tb.p};
    return SDH_OK;
  }
  std::vector<int64_t> run_off((size_t)W + 1, 0), wbase((size_t)W, 0);
  int64_t TW = 0;
  for (int r = 0; r < W; ++r) {
    run_off[(size_t)r + 1] = run_off[(size_t)r] + all[(size_t)r * xch::HDR];
    wbase[(size_t)r] = TW;
    TW += all[(size_t)r * xch::HDR + 1];
  }
  const int64_t N = run_off[(size_t)W];
  const size_t rows = (size_t)std::max<int64_t>(1, N);
  e->xg_q.ensure(rows);
  e->xg_key.ensure(rows);
  e->xg_ts.ensure(rows);
  e->xg_seq.ensure(rows);
  e->xg_tb.ensure(rows);
  e->xg_off.ensure((size_t)N + W);
  e->xg_words.ensure((size_t)std::max<int64_t>(1, TW));
  e->xg_keys.ensure(rows * kw);
  std::vector<std::vector<xch::Buf>> recv((size_t)W);
  for (int r = 0; r < W; ++r) {
    const int64_t o = run_off[(size_t)r], nr = all[(size_t)r * xch::HDR], wr = all[(size_t)r * xch::HDR + 1];
    recv[(size_t)r] = {{nullptr, e->xg_q.p + o, (size_t)nr * 8},          {nullptr, e->xg_key.p + o, (size_t)nr * 8},
                       {nullptr, e->xg_ts.p + o, (size_t)nr * 8},         {nullptr, e->xg_seq.p + o, (size_t)nr * 8},
                       {nullptr, e->xg_tb.p + o, (size_t)nr * 8},         {nullptr, e->xg_off.p + o + r, (size_t)(nr + 1) * 8},
                       {nullptr, e->xg_words.p + wbase[(size_t)r], (size_t)wr * 8},
                       {nullptr, e->xg_keys.p + o * kw, (size_t)nr * kw * 8}};
  }
  if (local) {  // rank 0's own run (RCCL: a self send / receive inside the gather)
    for (size_t i = 0; i < mine.size(); ++i)
      if (recv[0][i].bytes)
        HIPCHK(hipMemcpyAsync(recv[0][i].dst, mine[i].src, recv[0][i].bytes, hipMemcpyDeviceToDevice, e->stream));
    std::vector<std::vector<xch::Buf>> others(recv);
    others[0].clear();
    xcall([&] { xch::gather_bufs(e->comm, {}, others, e->stream); });
  } else {
    xcall([&] { xch::gather_bufs(e->comm, mine, recv, e->stream); });
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  table_clear(e);
  e->go_q.ensure(rows);
  e->go_key.ensure(rows);
  e->go_ts.ensure(rows);
  e->go_seq.ensure(rows);
  e->go_tb.ensure(rows);
  e->go_len.ensure((size_t)N + 1);
  e->go_off.ensure((size_t)N + 1);
  e->go_src.ensure(rows);
  e->go_pos.ensure(rows);
  e->go_temp.ensure(sdh_merge_temp_bytes(N));
  int64_t total = 0;
  HIPCHK(sdh_merge_runs(e->xg_keys.p, kw, run_off.data(), W, N, e->xg_q.p, e->xg_key.p, e->xg_ts.p, e->xg_seq.p,
                        e->xg_tb.p, e->xg_off.p, wbase.data(), e->go_pos.p, e->go_q.p, e->go_key.p, e->go_ts.p,
                        e->go_seq.p, e->go_tb.p, e->go_len.p, e->go_off.p, e->go_src.p, e->go_temp.p, e->go_temp.n,
                        &total, e->stream));
  if (total != TW) throw Error(SDH_E_DEVICE, "sdh_engine_gather: merged word count differs from the runs'");
  e->go_words.ensure((size_t)std::max<int64_t>(1, TW));
  HIPCHK(sdh_merge_words(e->go_src.p, e->go_off.p, N, e->xg_words.p, e->go_words.p, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (!host) {
    *out = sdh_matches{N, e->go_q.p, e->go_key.p, e->go_ts.p, e->go_off.p, e->go_words.p, e->go_seq.p, e->go_tb.p};
    return SDH_OK;
  }
  const size_t hn = (size_t)std::max<int64_t>(N, 1);
  e->ho_q.ensure(hn);
  e->ho_key.ensure(hn);
  e->ho_ts.ensure(hn);
  e->ho_seq.ensure(hn);
  e->ho_tb.ensure(hn);
  e->ho_off.ensure((size_t)N + 1);
  e->ho_words.ensure((size_t)std::max<int64_t>(TW, 1));
  const std::vector<std::tuple<void*, const void*, size_t>> cp = {
      {e->ho_q.p, e->go_q.p, (size_t)N * 8},     {e->ho_key.p, e->go_key.p, (size_t)N * 8},
      {e->ho_ts.p, e->go_ts.p, (size_t)N * 8},   {e->ho_seq.p, e->go_seq.p, (size_t)N * 8},
      {e->ho_tb.p, e->go_tb.p, (size_t)N * 8},   {e->ho_off.p, e->go_off.p, (size_t)(N + 1) * 8},
      {e->ho_words.p, e->go_words.p, (size_t)TW * 8}};
  for (const auto& c : cp)
    if (std::get<2>(c)) HIPCHK(hipMemcpyAsync(std::get<0>(c), std::get<1>(c), std::get<2>(c), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *out = sdh_matches{N, e->ho_q.p, e->ho_key.p, e->ho_ts.p, e->ho_off.p, e->ho_words.p, e->ho_seq.p, e->ho_tb.p};
  return SDH_OK;
}

// the absent states' timers due by t fire, with the next event's seq (sdh_engine_advance_time, and
// a chunk push before its first event)
void time_advance(sdh_engine* e, int64_t t) {
  if (!e->has_absent) return;
  HIPCHK(hipSetDevice(e->dev));
  StreamBatch B{};
  B.n = 0;
  B.stream = 0;
  B.n_attr = (int)e->prog.stream_types[0].size();
  B.seq_base = e->seq;
  B.prev_ts = e->prev_ts[0];
  e->work.clear();
  e->device_matches = 0;
  e->r_blocks_used = 0;
  e->r_matches = 0;
  e->r_placing = false;  // (the digest then reads no stale placed rows)
  e->g_dev_matches = 0;
  e->g_used = 0;
  e->dev_polled = false;
  e->last_n = 0;
  e->last_seq_base = e->seq;
  double ms = 0, bytes = 0;
  e->advance_to = t;
  try {
    launch_gen(e, 0, B, &ms, &bytes);
  } catch (const std::exception& ex) {
    e->advance_to = INT64_MIN;
    e->broken = ex.what();
    throw;
  }
  e->advance_to = INT64_MIN;
  if (!(e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) && e->g_dev_matches) {
    placed_to_table(e);
    append_gen(e, nullptr, 0, 0);
  }
}

// A chunk push (sdh_batch.chunk; include/siddhi_hip.h): per partition keyed on the stream, each
// event's same-key run start (PartitionStreamReceiver.receive(Event[]):214-239 -- runs of
// consecutive events with equal String.valueOf keys; an event with a null key is skipped and does
// not end a run), and per query the run table it reads (-1: none, -2: fan-out, by key position).
// Computed on the host from the key columns (copied back for a device-resident batch).
void chunk_begin(sdh_engine* e, int stream, const sdh_batch* b) {
  const int64_t n = b->n;
  const size_t nq = e->prog.q.size();
  std::vector<int32_t> qslot(std::max<size_t>(1, nq), -1), runs;
  int slots = 0;
  bool fan = false;
  for (const auto& pd : e->lp.parts) {
    int attr = -1;
    for (const auto& k : pd.keys)
      if (k.stream == stream) attr = (int)k.code[0].imm;
    if (attr < 0) {
      if (pd.fan(stream)) {
        fan = true;
        for (int pq : pd.queries) qslot[(size_t)pq] = -2;
      }
      continue;
    }
    for (int pq : pd.queries) qslot[(size_t)pq] = slots;
    const int type = e->lp.stream_types[stream][attr];
    const int w = attr_width(type);
    std::vector<uint8_t> col((size_t)n * w), nul;
    const bool has_nul = b->nulls && b->nulls[attr];
    if (has_nul) nul.resize((size_t)n);
    if (b->on_device) {
      d2h_sync(e, col.data(), b->cols[attr], col.size());
      if (has_nul) d2h_sync(e, nul.data(), b->nulls[attr], nul.size());
    } else {
      memcpy(col.data(), b->cols[attr], col.size());
      if (has_nul) memcpy(nul.data(), b->nulls[attr], nul.size());
    }
    runs.resize((size_t)(slots + 1) * n, 0);
    int32_t* r = runs.data() + (size_t)slots * n;
    int64_t prev = 0, start = 0;
    bool have = false;
    for (int64_t i = 0; i < n; ++i) {
      if (has_nul && nul[(size_t)i]) continue;
      int64_t raw;
      if (w == 8) memcpy(&raw, col.data() + (size_t)i * 8, 8);
      else if (w == 4) {
        int32_t v;
        memcpy(&v, col.data() + (size_t)i * 4, 4);
        raw = v;
      } else raw = col[(size_t)i];
      const int64_t k = kg::key_of_raw(type, raw);
      if (!have || k != prev) start = i;
      have = true;
      prev = k;
      r[i] = (int32_t)start;
    }
    ++slots;
  }
  e->ck_runs.ensure(std::max<size_t>(1, runs.size()));
  if (!runs.empty()) HIPCHK(hipMemcpy(e->ck_runs.p, runs.data(), runs.size() * 4, hipMemcpyHostToDevice));
  e->d_ck_qslot.ensure(qslot.size());
  HIPCHK(hipMemcpy(e->d_ck_qslot.p, qslot.data(), qslot.size() * 4, hipMemcpyHostToDevice));
  e->mt.max_run = std::max<int64_t>(e->mt.max_run, fan ? (int64_t)INT32_MAX : n);
}

int push_chunk(sdh_engine* e, int32_t stream, const sdh_batch* b) {
  if (stream < 0 || stream >= (int)e->prog.stream_types.size() || b->n_cols != (int)e->prog.stream_types[stream].size())
    throw Error(SDH_E_INVALID, "bad stream or batch");
  if (e->cfg.max_batch > 0 && b->n > e->cfg.max_batch) throw Error(SDH_E_INVALID, "batch larger than max_batch");
  if (b->n >= INT32_MAX) throw Error(SDH_E_INVALID, "a chunk of 2^31 events or more");
  if (b->n > 0) check_fan_strings(e, stream);
  HIPCHK(hipSetDevice(e->dev));
  int64_t t01[2];
  if (b->on_device) {
    d2h_sync(e, &t01[0], b->ts, 8);
    d2h_sync(e, &t01[1], b->ts + (b->n - 1), 8);
  } else {
    t01[0] = b->ts[0];
    t01[1] = b->ts[b->n - 1];
  }
  chunk_begin(e, stream, b);
  // InputHandler.send(Event[]):77-85: time moves once, to the last timestamp, before the chunk
  if (!e->started) {
    e->started = true;
    e->start_ts = t01[0];
  }
  time_advance(e, t01[1]);
  e->ck.active = true;
  e->mt.chunk_pushed = true;
  e->ck.first_seq = e->seq;
  e->ck.n = b->n;
  e->ck.stream = stream;
  try {
    do_push(e, stream, b);
  } catch (...) {
    e->ck.active = false;
    throw;
  }
  e->ck.active = false;
  return SDH_OK;
}

thread_local std::string g_create_error;

}  // namespace

extern "C" {

const char* sdh_version(void) { return "libsiddhi_hip 0.2 (gfx950: K_ratchet, K_chain, K_gen, K_seq; device R18 poll)"; }

int sdh_engine_create(const void* ir, size_t len, const sdh_config* cfg, sdh_engine** out) {
  if (!out) return SDH_E_INVALID;
  *out = nullptr;
  sdh_engine* e = new sdh_engine;
  int rc = guard(e, [&]() {
    if (cfg) e->cfg = *cfg;
    // sdh_config.debug: "NAME=VALUE;..." knobs (knobs.h), copied: the caller's string need not outlive
    // the call
    if (e->cfg.debug) {
      const std::string d(e->cfg.debug);
      size_t i = 0;
      while (i < d.size()) {
        size_t j = d.find(';', i);
        if (j == std::string::npos) j = d.size();
        const std::string kv = d.substr(i, j - i);
        const size_t eq = kv.find('=');
        if (!kv.empty()) e->knobs.emplace_back(kv.substr(0, eq), eq == std::string::npos ? "1" : kv.substr(eq + 1));
        i = j + 1;
      }
      e->cfg.debug = nullptr;
    }
    if (e->cfg.shard_world <= 0) e->cfg.shard_world = 1;
    e->dev = e->cfg.device;
    // the program is validated before any device call (a malformed blob is SDH_E_INVALID with or
    // without a GPU)
    e->prog = read_ir(ir, len);
    try {
      e->lp = kg::read_program(ir, len);
    } catch (const kg::LowerError& ex) {
      throw Error(SDH_E_INVALID, ex.what());
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
      (void)hipGetLastError();
      throw Error(SDH_E_DEVICE, "no HIP device (the engine has no CPU fallback)");
    }
    if (e->dev < 0 || e->dev >= ndev) throw Error(SDH_E_INVALID, fmt("device %d of %d", e->dev, ndev));
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipDeviceGetAttribute(&e->n_cu, hipDeviceAttributeMultiprocessorCount, e->dev));
    // tuning overrides for kernel experiments: K_ratchet LDS ring depth and waves per launch
    if (const char* v = sdh::knob("SDH_RATCHET_ML")) e->rML = std::max(4, atoi(v));
    if (const char* v = sdh::knob("SDH_RATCHET_WAVES")) e->r_waves = atof(v);
    if (const char* v = sdh::knob("SDH_XCD")) e->xcd = atoi(v) != 0;
    if (const char* v = sdh::knob("SDH_SLAB_LDS_SMALL")) e->slab_lds_small = std::max(64, atoi(v));
    e->out_rank = kg::output_ranks(e->lp);
    // plan selection per query: K_ratchet (2-state threshold ratchet) > K_chain (stream-state
    // chains) > K_gen (everything else: count, logical, sequences, partitions, general predicates)
    std::vector<std::pair<RatchetPlan, int>> rplans;
    std::vector<int> gen_qs;
    const bool no_ratchet = (e->cfg.flags & SDH_FLAG_NO_RATCHET) != 0;
    const bool force_gen = (e->cfg.flags & SDH_FLAG_FORCE_GEN) != 0;
    for (int qi = 0; qi < (int)e->prog.q.size(); ++qi) {
      // multi-GPU: unpartitioned queries are sharded by pattern set (query q on rank
      // q % world); a partition's queries run on every rank, each rank owning the keys that
      // key_shard maps to it (nfa_gen.hip: foreign keys' events are dropped at routing)
      if (e->lp.q[qi].partition < 0 && qi % e->cfg.shard_world != e->cfg.shard_rank) continue;
      Lowered L = force_gen ? Lowered() : lower_query(e->prog, qi);
      if (!L.ok) {
        gen_qs.push_back(qi);
        continue;
      }
      RatchetPlan rp = no_ratchet ? RatchetPlan() : ratchet_plan(L.cq);
      if (rp.ok) rplans.push_back({rp, qi});
      else e->lq.push_back(L);
    }
    int want = e->cfg.partials_per_inst > 0 ? e->cfg.partials_per_inst : 128;
    e->K = want <= 64 ? 1 : want <= 128 ? 2 : want <= 256 ? 4 : 8;
    e->pcap = 64 * e->K;
    int maxS = rplans.empty() ? 1 : 2;
    for (auto& L : e->lq) maxS = std::max(maxS, L.cq.n_states);
    e->rec_words = 2 + maxS;
    e->prev_ts.assign(e->prog.stream_types.size(), INT64_MIN);
    HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&e->h2d, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&e->ev0));
    HIPCHK(hipEventCreate(&e->ev1));
    HIPCHK(hipEventCreate(&e->ev_h0));
    HIPCHK(hipEventCreate(&e->ev_h1));
    for (auto& ev : e->ev_stage) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    e->d_q.ensure(std::max<size_t>(1, e->lq.size()));
    std::vector<ChainQuery> cqs;
    for (auto& L : e->lq) cqs.push_back(L.cq);
    if (!cqs.empty())
      HIPCHK(hipMemcpy(e->d_q.p, cqs.data(), cqs.size() * sizeof(ChainQuery), hipMemcpyHostToDevice));
    ensure_state(e);
    ratchet_build(e, rplans);
    gen_build(e, gen_qs);
    // R18 tables of the device match table: receiver rank per (query, stream), and per query its
    // state count and the stream of its last state (the trigger of a chain-plan match)
    const size_t nq_all = e->prog.q.size();
    if (nq_all >= ((size_t)1 << RANK_BITS)) throw Error(SDH_E_UNSUPPORTED, "more than 2^20 queries");
    // device ranks are out_rank + 1: rank 0 orders the absent states' timer matches before the
    // triggering event's own
    e->d_out_rank.ensure(std::max<size_t>(1, e->out_rank.size()));
    e->d_fan_rank.ensure(std::max<size_t>(1, e->out_rank.size()));
    if (!e->out_rank.empty()) {
      std::vector<int32_t> r1(e->out_rank.size()), fr(e->out_rank.size(), -1);
      for (size_t k = 0; k < r1.size(); ++k) r1[k] = e->out_rank[k] + 1;
      // fan-out (query, stream): the partition's first rank for that stream, and the query's rank
      // within it as a tiebreak below the key's junction-map position (the key-major order of
      // PartitionStreamReceiver.send(ComplexEvent))
      const size_t ns = e->prog.stream_types.size();
      for (const auto& pd : e->lp.parts)
        for (const auto& f : pd.fanout) {
          int base = INT32_MAX;
          for (int pq : pd.queries) base = std::min(base, e->out_rank[(size_t)pq * ns + f.stream]);
          for (int pq : pd.queries) {
            fr[(size_t)pq * ns + f.stream] = e->out_rank[(size_t)pq * ns + f.stream] - base;
            r1[(size_t)pq * ns + f.stream] = base + 1;
          }
        }
      HIPCHK(hipMemcpy(e->d_out_rank.p, r1.data(), r1.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_fan_rank.p, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
      // chunk delivery (matches.hip chunk_keys_kernel): a query's junction subscriber rank (+1) --
      // its partition's first rank on the stream -- and its rank inside the partition
      e->ck_major = r1;
      e->ck_minor.assign(r1.size(), 0);
      for (const auto& pd : e->lp.parts)
        for (size_t st = 0; st < ns; ++st) {
          int base = INT32_MAX;
          for (int pq : pd.queries) base = std::min(base, e->out_rank[(size_t)pq * ns + st]);
          for (int pq : pd.queries) {
            e->ck_major[(size_t)pq * ns + st] = base + 1;
            e->ck_minor[(size_t)pq * ns + st] = e->out_rank[(size_t)pq * ns + st] - base;
          }
        }
      e->d_ck_major.ensure(r1.size());
      e->d_ck_minor.ensure(r1.size());
      HIPCHK(hipMemcpy(e->d_ck_major.p, e->ck_major.data(), r1.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_ck_minor.p, e->ck_minor.data(), r1.size() * 4, hipMemcpyHostToDevice));
    }
    // direct placement cells: a stream qualifies when its K_ratchet groups, each in lane order, are
    // consecutive runs of its K_ratchet queries in receiver-rank order (a placed push has no other
    // producer); cell = the group's run position
    {
      const size_t ns = e->prog.stream_types.size();
      e->place_cells.assign(ns, 0);
      for (auto& g : e->rg) g.cell = -1;
      for (size_t st = 0; st < ns; ++st) {
        std::vector<int> gs;
        bool gated = false;  // (K_gate writes records, not placed rows)
        for (int g = 0; g < (int)e->rg.size(); ++g)
          if (e->rg[g].stream == (int)st && e->rg[g].n_lanes > 0) {
            gs.push_back(g);
            gated |= e->rg[g].n_g > 0;
          }
        if (gs.empty() || gated) continue;
        auto rk = [&](int g, int l) { return e->out_rank[(size_t)e->rg[g].qid[l] * ns + st]; };
        std::sort(gs.begin(), gs.end(), [&](int a, int b) { return rk(a, 0) < rk(b, 0); });
        std::vector<int> ranks;
        for (int g : gs)
          for (int l = 0; l < e->rg[g].n_lanes; ++l) ranks.push_back(rk(g, l));
        bool ok = true;
        for (size_t k = 1; k < ranks.size(); ++k) ok = ok && ranks[k - 1] < ranks[k];
        if (!ok) continue;
        for (size_t c = 0; c < gs.size(); ++c) e->rg[gs[c]].cell = (int)c;
        e->place_cells[st] = (int)gs.size();
      }
      if (!e->rg.empty())
        HIPCHK(hipMemcpy(e->d_rg.p, e->rg.data(), e->rg.size() * sizeof(RatchetGroup), hipMemcpyHostToDevice));
    }
    std::vector<int32_t> qinfo(std::max<size_t>(1, 2 * nq_all), 0);
    for (size_t q = 0; q < nq_all; ++q) {
      qinfo[2 * q] = (int32_t)e->prog.q[q].st.size();
      qinfo[2 * q + 1] = e->prog.q[q].st.empty() ? 0 : e->prog.q[q].st.back().stream;
    }
    e->d_qinfo.ensure(qinfo.size());
    HIPCHK(hipMemcpy(e->d_qinfo.p, qinfo.data(), qinfo.size() * 4, hipMemcpyHostToDevice));
    for (size_t q = 0; q < nq_all; ++q) e->cw = std::max(e->cw, 2 + qinfo[2 * q]);
    return SDH_OK;
  });
  if (rc != SDH_OK) {
    g_create_error = e->err;
    delete e;
    return rc;
  }
  *out = e;
  return SDH_OK;
}

int sdh_engine_push(sdh_engine* e, int32_t stream, const sdh_batch* b) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    if (b && b->chunk && b->n > 1) return push_chunk(e, stream, b);
    return do_push(e, stream, b);
  });
}

int sdh_engine_reserve(sdh_engine* e, int64_t bytes) {
  if (!e || bytes < 0) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    HIPCHK(hipSetDevice(e->dev));
    if (e->ssets.empty() || bytes == 0) return SDH_OK;
    const size_t per = (size_t)bytes / e->ssets.size();
    for (auto& ss : e->ssets)
      if (ss->arena_bytes < per && !ss->add_chunk(((per - ss->arena_bytes) + 4095) & ~(size_t)4095))
        throw Error(SDH_E_CAPACITY, fmt("device memory exhausted reserving %.1f GB for the sparse state", bytes / 1e9));
    return SDH_OK;
  });
}

int sdh_engine_reserve_keys(sdh_engine* e, int64_t keys) {
  if (!e || keys < 0) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    HIPCHK(hipSetDevice(e->dev));
    if (keys == 0) return SDH_OK;
    for (auto& r : e->routes)
      if (r && keys > r->max_keys)
        throw Error(SDH_E_INVALID, fmt("reserve_keys(%lld) beyond gen_max_keys (%lld)", (long long)keys,
                                       (long long)r->max_keys));
    // the same growth calls a push makes when its batch brings new keys (a prefix copy of held state)
    for (auto& gs : e->gsets)
      if (gs->partition >= 0 && gs->n_groups > 0) gen_grow(e, *gs, keys);
    for (auto& ps : e->psets) part_grow(e, *ps, keys);
    for (auto& ss : e->ssets) slab_grow_keys(e, *ss, keys);
    return SDH_OK;
  });
}

int sdh_engine_poll_compact_ex(sdh_engine* e, int32_t device, sdh_matches_compact_ex* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() { return do_poll_compact_ex(e, out, device != 0); });
}

int sdh_engine_set_comm(sdh_engine* e, sdh_comm* c) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    if (c && xch::device(c) != e->dev)
      throw Error(SDH_E_INVALID, fmt("communicator on device %d, engine on device %d", xch::device(c), e->dev));
    e->comm = c;
    return SDH_OK;
  });
}

int sdh_engine_push_bcast(sdh_engine* e, int32_t stream, const sdh_batch* b, int32_t root) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    return do_push_bcast(e, stream, b, root);
  });
}

int sdh_engine_gather(sdh_engine* e, int32_t device, sdh_matches* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    return do_gather(e, out, device == 0);
  });
}

int sdh_engine_flush(sdh_engine* e) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    HIPCHK(hipStreamSynchronize(e->stream));
    return SDH_OK;
  });
}

int sdh_engine_start(sdh_engine* e, int64_t t) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    if (e->started) throw Error(SDH_E_INVALID, "the engine has already started");
    e->started = true;
    e->start_ts = t;
    return SDH_OK;
  });
}

// Time passes to t with no event: every absent state's scheduler fires what falls due (the timer
// thread of a live runtime, Scheduler.java:258-287). Its matches join the device table like a
// push's, ordered by (timer time, query, fire order) before the next event's.
int sdh_engine_advance_time(sdh_engine* e, int64_t t) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    if (!e->started) {
      e->started = true;
      e->start_ts = t;
    }
    time_advance(e, t);
    return SDH_OK;
  });
}

int sdh_engine_pending_matches(sdh_engine* e, int64_t* n) {
  if (!e || !n) return SDH_E_INVALID;
  *n = e->mt.n + ((e->cfg.flags & SDH_FLAG_DEVICE_MATCHES) && !e->dev_polled
                       ? e->device_matches + e->r_matches + e->g_dev_matches : 0);
  return SDH_OK;
}

int sdh_engine_poll(sdh_engine* e, sdh_matches* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() { return do_poll(e, out, true); });
}

int sdh_engine_poll_device(sdh_engine* e, sdh_matches* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() { return do_poll(e, out, false); });
}

int sdh_engine_poll_compact(sdh_engine* e, int32_t device, sdh_matches_compact* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() { return do_poll_compact(e, out, device != 0); });
}

// keys a partition has seen so far (its routing table's dense ids)
int64_t route_keys(sdh_engine* e, int partition) {
  if (partition < 0 || partition >= (int)e->routes.size() || !e->routes[partition]) return 0;
  int32_t nk = 0;
  d2h_sync(e, &nk, e->routes[partition]->n_keys.p, 4);
  return nk;
}

// Live partials of K_gen arenas, K_part tables and K_seq windows: entries of the pending lists of
// non-start states (oracle_live_partials counts every pending list, the start state's seed included)
int64_t device_live_partials(sdh_engine* e) {
  DevBuf<unsigned long long> acc;
  acc.ensure(1);
  HIPCHK(hipMemsetAsync(acc.p, 0, 8, e->stream));
  DevBuf<int32_t> d_gseq;
  if (!e->group_seq.empty()) {
    d_gseq.ensure(e->group_seq.size());
    HIPCHK(hipMemcpy(d_gseq.p, e->group_seq.data(), e->group_seq.size() * 4, hipMemcpyHostToDevice));
  }
  for (auto& up : e->gsets) {
    auto& gs = *up;
    if (!gs.a32.p || gs.n_groups == 0) continue;
    const int64_t blocks = gs.partition < 0 ? gs.n_groups : std::min(gs.key_cap, route_keys(e, gs.partition)) * gs.n_groups;
    HIPCHK(sdh_live_gen(gs.a32.p, e->gB32, blocks, gs.n_groups, gs.group_base, e->d_lane_q.p, d_gseq.p, e->d_gq.p, acc.p,
                        e->stream));
  }
  for (auto& up : e->psets) {
    auto& ps = *up;
    if (!ps.st.p || ps.key_cap == 0) continue;
    const int64_t nk = std::min(ps.key_cap, route_keys(e, ps.partition));
    HIPCHK(sdh_live_part(ps.st.p, ps.cur.p, nk, ps.n_groups, ps.key_cap * ps.n_groups, ps.bw(), acc.p, e->stream));
  }
  for (int s = 0; s < (int)e->seq_tail.size(); ++s) {
    std::vector<int32_t> gl;
    for (int g = 0; g < (int)e->group_seq.size(); ++g)
      if (e->group_seq[g] > 0 && e->gq[e->group_tmpl[g]].st[0].stream == s) gl.push_back(g);
    if (gl.empty() || e->seq_tail_len[s] <= 0) continue;
    DevBuf<int32_t> d_gl;
    d_gl.ensure(gl.size());
    HIPCHK(hipMemcpy(d_gl.p, gl.data(), gl.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(sdh_live_seq(e->seq_tail[s].p, e->seq_tail_len[s], s, d_gl.p, (int)gl.size(), e->d_lane_q.p,
                        e->d_group_tmpl.p, e->d_gq.p, acc.p, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));  // (d_gl is freed at scope end)
  }
  unsigned long long v = 0;
  d2h_sync(e, &v, acc.p, 8);
  return (int64_t)v;
}

// Test diagnostic: (records, order-independent hash) of the last push's K_ratchet records as the
// kernel wrote them, in either output mode (matches.hip digest_ratchet_kernel)
int sdh_engine_debug_digest(sdh_engine* e, uint64_t* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() {
    out[0] = out[1] = 0;
    DevBuf<unsigned long long> acc;
    acc.ensure(2);
    HIPCHK(hipMemsetAsync(acc.p, 0, 16, e->stream));
    if (e->r_placing)  // the last push placed its matches: its compact rows
      HIPCHK(sdh_digest_compact(e->pc_rows.p, e->cw, e->r_place_row0, e->r_matches, e->seq_ref, acc.p, e->stream));
    else
      HIPCHK(sdh_digest_ratchet(e->d_rmatch.p, e->r_blk_recs, e->r_wide, e->d_blk_count.p, e->d_blk_group.p,
                                e->d_blk_side.p, e->d_rg.p, e->r_seq_base, (int)e->r_blk_taken, acc.p, e->stream));
    d2h_sync(e, out, acc.p, 16);
    return SDH_OK;
  });
}

// The last push's device records (SDH_FLAG_DEVICE_MATCHES; formats: include/siddhi_hip.h sdh_records)
int sdh_engine_poll_records(sdh_engine* e, sdh_records* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    *out = sdh_records{};
    if (!(e->cfg.flags & SDH_FLAG_DEVICE_MATCHES))
      throw Error(SDH_E_INVALID, "sdh_engine_poll_records needs SDH_FLAG_DEVICE_MATCHES (use sdh_engine_poll)");
    out->seq_base = e->last_seq_base;
    out->n_events = e->last_n;
    if (e->r_blocks_used > 0 && !e->r_placing) {
      if (e->d_rlane_q.n < e->rg.size() * WAVE) {
        std::vector<int32_t> lq(e->rg.size() * WAVE, -1);
        for (size_t g = 0; g < e->rg.size(); ++g)
          for (int l = 0; l < e->rg[g].n_lanes; ++l) lq[g * WAVE + l] = e->rg[g].qid[l];
        e->d_rlane_q.ensure(lq.size());
        HIPCHK(hipMemcpy(e->d_rlane_q.p, lq.data(), lq.size() * 4, hipMemcpyHostToDevice));
      }
      out->r_n = e->r_matches;
      out->r_blocks = e->r_blocks_used;
      out->r_bytes = (int64_t)e->r_rec_bytes;
      out->r_base = e->d_rmatch.p;
      out->r_count = e->d_blk_count.p;
      out->r_side = e->d_blk_side.p;
      out->r_group = e->d_blk_group.p;
      out->r_lane_query = e->d_rlane_q.p;
      out->r_format = e->r_rec4 ? SDH_REC_4 : e->r_wide ? SDH_REC_16 : SDH_REC_8;
      out->r_blk_bytes = e->r_blk_recs * 8 * (e->r_wide ? 2 : 1);
    }
    if (e->g_dev_matches > 0) {
      upload_qkeys(e);
      out->f_n = e->g_dev_matches;
      out->f_words = e->g_used;
      out->f_base = e->g_out.p;
      out->f_query_keys = e->d_qkeys.p;
    }
    if (e->device_matches > 0) {
      const int64_t ni = (int64_t)e->work.size();
      std::vector<int64_t> so(ni);
      for (int64_t i = 0; i < ni; ++i) so[i] = e->work[i].seg_off;
      e->d_seg_off.ensure(ni);
      HIPCHK(hipMemcpy(e->d_seg_off.p, so.data(), ni * 8, hipMemcpyHostToDevice));
      out->c_n = e->device_matches;
      out->c_items = ni;
      out->c_words = e->rec_words;
      out->c_base = e->d_match.p;
      out->c_off = e->d_seg_off.p;
      out->c_count = e->d_seg_count.p;
    }
    out->n = out->r_n + out->f_n + out->c_n;
    e->dev_polled = true;
    return SDH_OK;
  });
}

int sdh_engine_records_compact(sdh_engine* e, int32_t* rows, int64_t cap, int32_t width, int64_t* n) {
  if (!e || !n || width < 4) return SDH_E_INVALID;
  return guard(e, [&]() {
    check_usable(e);
    *n = 0;
    if (!(e->cfg.flags & SDH_FLAG_DEVICE_MATCHES))
      throw Error(SDH_E_INVALID, "sdh_engine_records_compact needs SDH_FLAG_DEVICE_MATCHES");
    const int nb = e->r_placing ? 0 : e->r_blocks_used;
    if (nb <= 0) return SDH_OK;
    *n = e->r_matches;
    if (!rows) return SDH_OK;
    if (cap < e->r_matches) throw Error(SDH_E_CAPACITY, fmt("%lld rows need room for %lld", (long long)cap, (long long)e->r_matches));
    e->d_rrow_off.ensure((size_t)nb + 1);
    e->d_rrow_tmp.ensure(sdh_ratchet_compact_temp(nb));
    HIPCHK(sdh_ratchet_compact(e->d_rmatch.p, e->r_blk_recs, e->r_wide, e->d_blk_count.p, e->d_blk_group.p,
                               e->d_blk_side.p, e->d_rg.p, e->r_seq_base, nb, e->d_rrow_off.p, e->d_rrow_tmp.p,
                               e->d_rrow_tmp.n, width, rows, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return SDH_OK;
  });
}

int sdh_engine_push_stats(sdh_engine* e, double* last_kernel_ms, double* last_kernel_bytes) {
  if (!e || !last_kernel_ms || !last_kernel_bytes) return SDH_E_INVALID;
  *last_kernel_ms = e->stats.last_kernel_ms;  // (host-side values: no device work, no sync)
  *last_kernel_bytes = e->stats.last_kernel_bytes;
  return SDH_OK;
}

int sdh_engine_stats(sdh_engine* e, sdh_stats* out) {
  if (!e || !out) return SDH_E_INVALID;
  return guard(e, [&]() {
    const size_t nq = e->lq.size();
    std::vector<InstHeader> h[2];
    int64_t live = 0;
    for (int b = 0; b < 2 && nq; ++b) {
      h[b].resize(nq);
      d2h_sync(e, h[b].data(), e->d_hdr[b].p, nq * sizeof(InstHeader));
    }
    for (size_t q = 0; q < nq; ++q) live += h[e->cur[q]][q].n_live;
    const size_t ng = e->rg.size();
    for (int b = 0; b < 2 && ng; ++b) {
      std::vector<RatchetState> rs(ng);
      d2h_sync(e, rs.data(), e->d_rst[b].p, ng * sizeof(RatchetState));
      for (size_t g = 0; g < ng; ++g)
        if (e->rcur[g] == b)
          for (int l = 0; l < e->rg[g].n_lanes; ++l) live += rs[g].n[l];
    }
    for (auto& ss : e->ssets) live += slab_live_partials(e, *ss);
    live += device_live_partials(e);
    e->stats.live_partials = live;
    e->stats.pool_regrows = e->gen_regrows;
    e->stats.last_slab_items = e->slab_items;
    // queries per plan: K_ratchet, K_gate, K_chain, K_part, K_slab, K_seq, K_gen
    for (auto& c : e->stats.plan_queries) c = 0;
    for (const auto& g : e->rg) e->stats.plan_queries[g.n_g ? 1 : 0] += g.n_lanes;
    e->stats.plan_queries[2] = (int64_t)e->lq.size();
    auto lanes = [&](int g) {
      int64_t c = 0;
      for (int l = 0; l < WAVE; ++l) c += e->lane_q[(size_t)g * WAVE + l] >= 0 ? 1 : 0;
      return c;
    };
    for (const auto& ps : e->psets)
      for (int g = ps->group_base; g < ps->group_base + ps->n_groups; ++g) e->stats.plan_queries[3] += lanes(g);
    for (const auto& ss : e->ssets)
      for (int g = ss->group_base; g < ss->group_base + ss->n_groups; ++g) e->stats.plan_queries[4] += lanes(g);
    for (const auto& gs : e->gsets)
      for (int g = gs->group_base; g < gs->group_base + gs->n_groups; ++g)
        e->stats.plan_queries[(size_t)g < e->group_seq.size() && e->group_seq[g] > 0 ? 5 : 6] += lanes(g);
    *out = e->stats;
    return SDH_OK;
  });
}

// snapshot: [magic][version][n_q][pcap][gB32][gB64][R][N][LC][started][start_ts][seq][n_streams][prev_ts...]
// then per query
// header + table, ratchet deques, K_gen arenas + key tables, K_seq tails
constexpr int64_t SNAP_MAGIC = 0x5344485350415254LL;
constexpr int64_t SNAP_VERSION = 8;
// Device memory of the sparse K_slab state: the live blocks' bytes, the slab's reserved bytes (live
// blocks, not yet reclaimed superseded ones, and free room) and the directory's
int sdh_engine_state_bytes(sdh_engine* e, int64_t* live_bytes, int64_t* reserved_bytes, int64_t* dir_bytes) {
  if (!e) return SDH_E_INVALID;
  return guard(e, [&]() {
    int64_t lb = 0, rb = 0, db = 0;
    DevBuf<unsigned long long> acc;
    acc.ensure(1);
    for (auto& up : e->ssets) {
      auto& ss = *up;
      HIPCHK(hipMemsetAsync(acc.p, 0, 8, e->stream));
      HIPCHK(sdh_slab_live_words(ss.dir.p, ss.key_cap * ss.n_groups, ss.n_groups, ss.d_group_ew.p, acc.p, e->stream));
      unsigned long long w = 0;
      HIPCHK(hipMemcpyAsync(&w, acc.p, 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      lb += (int64_t)w * 4;
      for (int64_t c : ss.cap) rb += c * 4;
      db += ss.key_cap * ss.n_groups * 8;
    }
    if (live_bytes) *live_bytes = lb;
    if (reserved_bytes) *reserved_bytes = rb;
    if (dir_bytes) *dir_bytes = db;
    return SDH_OK;
  });
}

int sdh_engine_set_strings(sdh_engine* e, int64_t n, const int32_t* ids, const int32_t* java_hash,
                           const int32_t* utf16_len) {
  if (!e || n < 0 || (n > 0 && (!ids || !java_hash || !utf16_len))) return SDH_E_INVALID;
  return guard(e, [&]() {
    for (int64_t i = 0; i < n; ++i) {
      if (utf16_len[i] < 0) throw Error(SDH_E_INVALID, "negative string length");
      e->str_info[ids[i]] = {java_hash[i], (int64_t)utf16_len[i]};
    }
    return SDH_OK;
  });
}

int sdh_engine_snapshot(sdh_engine* e, void** blob, size_t* len) {
  if (!e || !blob || !len) return SDH_E_INVALID;
  return guard(e, [&]() {
    HIPCHK(hipStreamSynchronize(e->stream));
    const size_t nq = e->lq.size();
    const size_t tbl = (size_t)NF * e->pcap;
    std::vector<int64_t> w{SNAP_MAGIC, SNAP_VERSION, (int64_t)nq, e->pcap, e->gB32, e->gB64,
                           e->gsz.R, e->gsz.N, e->gsz.LC, e->started ? 1 : 0, e->start_ts, e->seq,
                           (int64_t)e->prev_ts.size()};
    w.insert(w.end(), e->prev_ts.begin(), e->prev_ts.end());
    for (size_t q = 0; q < nq; ++q) {
      InstHeader h;
      HIPCHK(hipMemcpy(&h, e->d_hdr[e->cur[q]].p + q, sizeof h, hipMemcpyDeviceToHost));
      w.push_back(h.seed_alive);
      w.push_back(h.n_live);
      size_t o = w.size();
      w.resize(o + tbl);
      HIPCHK(hipMemcpy(&w[o], e->d_part[e->cur[q]].p + q * tbl, tbl * 8, hipMemcpyDeviceToHost));
    }
    // K_ratchet deques: per group, per lane: n then n x (ts0, seq, key)
    const size_t ng = e->rg.size();
    w.push_back((int64_t)ng);
    for (size_t g = 0; g < ng; ++g) {
      const int b = e->rcur[g];
      RatchetState rs;
      HIPCHK(hipMemcpy(&rs, e->d_rst[b].p + g, sizeof rs, hipMemcpyDeviceToHost));
      std::vector<int64_t> t(e->rsmax * WAVE), sq(e->rsmax * WAVE), ky(e->rsmax * WAVE);
      const size_t o = g * e->rsmax * WAVE;
      HIPCHK(hipMemcpy(t.data(), e->d_rts[b].p + o, t.size() * 8, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(sq.data(), e->d_rsq[b].p + o, sq.size() * 8, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(ky.data(), e->d_rky[b].p + o, ky.size() * 8, hipMemcpyDeviceToHost));
      for (int l = 0; l < WAVE; ++l) {
        w.push_back(rs.n[l]);
        for (int i = 0; i < rs.n[l]; ++i) {
          w.push_back(t[i * WAVE + l]);
          w.push_back(sq[i * WAVE + l]);
          w.push_back(ky[i * WAVE + l]);
        }
      }
    }
    // K_gen sets: instance arenas (Snapshotable state of every pre-processor of every instance)
    // and, for partitions, the key table (PartitionRuntime's key -> instance map)
    w.push_back((int64_t)e->gsets.size());
    auto put_dev = [&](const void* dptr, size_t bytes) {
      const size_t o = w.size();
      w.resize(o + (bytes + 7) / 8);
      if (bytes) HIPCHK(hipMemcpy(&w[o], dptr, bytes, hipMemcpyDeviceToHost));
    };
    for (auto& up : e->gsets) {
      auto& gs = *up;
      const int64_t blocks = gs.partition < 0 ? gs.n_groups : gs.key_cap * gs.n_groups;
      w.push_back(gs.partition);
      w.push_back(gs.key_cap);
      w.push_back(blocks);
      put_dev(gs.a32.p, (size_t)blocks * e->gB32 * 64 * 4);
      put_dev(gs.a64.p, (size_t)blocks * e->gB64 * 64 * 8);
    }
    // partition key tables (PartitionRuntime's key -> instance map)
    w.push_back((int64_t)e->routes.size());
    for (auto& rp : e->routes) {
      w.push_back(rp ? 1 : 0);
      if (!rp) continue;
      const size_t slots = (size_t)rp->tmask + 2;
      w.push_back((int64_t)slots);
      put_dev(rp->tkey.p, slots * 8);
      put_dev(rp->tid.p, slots * 4);
      put_dev(rp->n_keys.p, 4);
      put_dev(rp->key_of_id.p, (size_t)rp->max_keys * 8);
      // fan-out partitions: the keys' creation order (the junction maps' insertion order)
      w.push_back(rp->kkind);
      w.push_back(rp->nk_seen);
      w.push_back((int64_t)rp->korder_kid.size());
      for (size_t j = 0; j < rp->korder_kid.size(); ++j) {
        w.push_back(rp->korder_kid[j]);
        w.push_back(rp->korder_key[j]);
      }
    }
    // K_part tables: both buffers and the per-key selector
    w.push_back((int64_t)e->psets.size());
    for (auto& pp : e->psets) {
      auto& ps = *pp;
      w.push_back(ps.partition);
      w.push_back(ps.kind);
      w.push_back(ps.cap);
      w.push_back(ps.key_cap);
      put_dev(ps.st.p, (size_t)2 * ps.key_cap * ps.n_groups * ps.bw() * 64 * 8);
      put_dev(ps.cur.p, (size_t)ps.key_cap * 4);
    }
    // K_seq: each stream's tail (the only state its windowed sequences carry between pushes)
    w.push_back((int64_t)e->seq_tail.size());
    for (size_t st = 0; st < e->seq_tail.size(); ++st) {
      w.push_back(e->seq_tail_len[st]);
      put_dev(e->seq_tail[st].p, SEQ_TMAX * SEQ_TW * 8);
    }
    // K_slab: the live blocks packed into one ring, the directory pointing into it, the counters
    w.push_back((int64_t)e->ssets.size());
    for (auto& up : e->ssets) {
      auto& ss = *up;
      const int64_t n_dir = ss.key_cap * ss.n_groups;
      DevBuf<unsigned long long> acc, ph, pt;
      acc.ensure(1);
      ph.ensure(1);
      pt.ensure(1);
      HIPCHK(hipMemset(acc.p, 0, 8));
      HIPCHK(hipMemset(ph.p, 0, 8));
      HIPCHK(hipMemset(pt.p, 0, 8));
      HIPCHK(sdh_slab_live_words(ss.dir.p, n_dir, ss.n_groups, ss.d_group_ew.p, acc.p, e->stream));
      unsigned long long words = 0;
      HIPCHK(hipMemcpyAsync(&words, acc.p, 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      DevBuf<uint64_t> dcopy;
      DevBuf<uint32_t> packed;
      dcopy.ensure(std::max<int64_t>(1, n_dir));
      packed.ensure(std::max<size_t>(1, (size_t)words));
      if (n_dir) HIPCHK(hipMemcpy(dcopy.p, ss.dir.p, n_dir * 8, hipMemcpyDeviceToDevice));
      DevBuf<uint32_t*> pr;
      DevBuf<int64_t> pc;
      pr.ensure(1);
      pc.ensure(1);
      const int64_t pcap = std::max<int64_t>(4, (int64_t)words);
      HIPCHK(hipMemcpy(pr.p, &packed.p, sizeof(uint32_t*), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(pc.p, &pcap, 8, hipMemcpyHostToDevice));
      if (words && !slab_move_raw(e, ss, dcopy.p, ss.d_ring.p, ss.d_cap.p, ss.tail.p, ss.nsub,
                                  std::vector<unsigned long long>(ss.nsub, ~0ull), {}, pr.p, pc.p, ph.p, pt.p, 1))
        throw Error(SDH_E_DEVICE, "K_slab snapshot: packing failed");
      w.push_back(ss.partition);
      w.push_back(ss.key_cap);
      w.push_back(ss.n_groups);
      w.push_back(ss.lds_words);
      w.push_back((int64_t)words);
      put_dev(dcopy.p, (size_t)n_dir * 8);
      put_dev(packed.p, (size_t)words * 4);
      put_dev(ss.live.p, 256 * 8);
    }
    *len = w.size() * 8;
    *blob = malloc(*len);
    memcpy(*blob, w.data(), *len);
    return SDH_OK;
  });
}

int sdh_engine_restore(sdh_engine* e, const void* blob, size_t len) {
  if (!e || !blob) return SDH_E_INVALID;
  return guard(e, [&]() {
    const int64_t* w = (const int64_t*)blob;
    size_t nw = len / 8, i = 0;
    auto nx = [&]() {
      if (i >= nw) throw Error(SDH_E_INVALID, "snapshot truncated");
      return w[i++];
    };
    if (nx() != SNAP_MAGIC) throw Error(SDH_E_INVALID, "bad snapshot magic");
    if (nx() != SNAP_VERSION) throw Error(SDH_E_INVALID, "snapshot of another format version");
    const size_t nq = (size_t)nx();
    if (nq != e->lq.size() || nx() != e->pcap) throw Error(SDH_E_INVALID, "snapshot of a different program");
    const int64_t b32 = nx(), b64 = nx();
    kg::Sizing sz;
    sz.R = (int)nx();
    sz.N = (int)nx();
    sz.LC = (int)nx();
    if (sz.R < 1 || sz.R > kg::GMAXPOOL || sz.N < 1 || sz.N > kg::GMAXPOOL || sz.LC < 1 || sz.LC > (1 << 16))
      throw Error(SDH_E_INVALID, "bad snapshot K_gen pool sizing");
    // the snapshot's pools may have grown past this engine's: take its sizing (arenas are loaded below)
    if (sz.R != e->gsz.R || sz.N != e->gsz.N || sz.LC != e->gsz.LC) gen_relayout(e, sz, false);
    if (b32 != e->gB32 || b64 != e->gB64)
      throw Error(SDH_E_INVALID, "snapshot of a different K_gen arena layout (another build or pool sizing)");
    e->started = nx() != 0;  // the runtime's start time (absent states' schedules)
    e->start_ts = nx();
    e->seq = nx();
    const size_t ns = (size_t)nx();
    if (ns != e->prev_ts.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    for (auto& t : e->prev_ts) t = nx();
    const size_t tbl = (size_t)NF * e->pcap;
    for (size_t q = 0; q < nq; ++q) {
      InstHeader h{(int32_t)nx(), (int32_t)nx(), 0, 0};
      if (i + tbl > nw) throw Error(SDH_E_INVALID, "snapshot truncated");
      HIPCHK(hipMemcpy(e->d_hdr[e->cur[q]].p + q, &h, sizeof h, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_part[e->cur[q]].p + q * tbl, &w[i], tbl * 8, hipMemcpyHostToDevice));
      i += tbl;
    }
    const size_t ng = (size_t)nx();
    if (ng != e->rg.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    // deques in snapshot order; the persisted capacity grows to the longest one first
    std::vector<size_t> at(ng);
    int64_t longest = 0;
    for (size_t g = 0; g < ng; ++g) {
      at[g] = i;
      for (int l = 0; l < WAVE; ++l) {
        const int64_t nl = nx();
        if (nl < 0 || nl > ((int64_t)1 << 26) || i + 3 * (size_t)nl > nw)
          throw Error(SDH_E_INVALID, "bad snapshot deque length");
        longest = std::max(longest, nl);
        i += 3 * (size_t)nl;
      }
    }
    ratchet_grow_rsmax(e, longest);
    const size_t i_end = i;
    for (size_t g = 0; g < ng; ++g) {
      i = at[g];
      const int b = e->rcur[g];
      RatchetState rs{};
      std::vector<int64_t> t(e->rsmax * WAVE, 0), sq(e->rsmax * WAVE, 0), ky(e->rsmax * WAVE, 0);
      for (int l = 0; l < WAVE; ++l) {
        const int64_t nl = nx();
        rs.n[l] = (int32_t)nl;
        for (int i = 0; i < nl; ++i) {
          t[i * WAVE + l] = nx();
          sq[i * WAVE + l] = nx();
          ky[i * WAVE + l] = nx();
        }
      }
      const size_t o = g * e->rsmax * WAVE;
      HIPCHK(hipMemcpy(e->d_rst[b].p + g, &rs, sizeof rs, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_rts[b].p + o, t.data(), t.size() * 8, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_rsq[b].p + o, sq.data(), sq.size() * 8, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(e->d_rky[b].p + o, ky.data(), ky.size() * 8, hipMemcpyHostToDevice));
    }
    i = i_end;
    if ((size_t)nx() != e->gsets.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    auto get_dev = [&](void* dptr, size_t bytes) {
      const size_t nw8 = (bytes + 7) / 8;
      if (i + nw8 > nw) throw Error(SDH_E_INVALID, "snapshot truncated");
      if (bytes) HIPCHK(hipMemcpy(dptr, &w[i], bytes, hipMemcpyHostToDevice));
      i += nw8;
    };
    for (auto& up : e->gsets) {
      auto& gs = *up;
      if (nx() != gs.partition) throw Error(SDH_E_INVALID, "snapshot of a different program");
      const int64_t key_cap = nx(), blocks = nx();
      if (gs.partition >= 0) {
        gen_grow(e, gs, key_cap);
        if (gs.key_cap != key_cap) throw Error(SDH_E_INVALID, "snapshot key capacity mismatch");
      }
      const int64_t want_blocks = gs.partition < 0 ? gs.n_groups : gs.key_cap * gs.n_groups;
      if (blocks != want_blocks) throw Error(SDH_E_INVALID, "snapshot arena size mismatch");
      get_dev(gs.a32.p, (size_t)blocks * e->gB32 * 64 * 4);
      get_dev(gs.a64.p, (size_t)blocks * e->gB64 * 64 * 8);
    }
    if ((size_t)nx() != e->routes.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    for (auto& rp : e->routes) {
      if (nx() != (rp ? 1 : 0)) throw Error(SDH_E_INVALID, "snapshot of a different program");
      if (!rp) continue;
      const size_t slots = (size_t)nx();
      if (slots != (size_t)rp->tmask + 2) throw Error(SDH_E_INVALID, "snapshot key table mismatch");
      get_dev(rp->tkey.p, slots * 8);
      get_dev(rp->tid.p, slots * 4);
      get_dev(rp->n_keys.p, 4);
      get_dev(rp->key_of_id.p, (size_t)rp->max_keys * 8);
      rp->kkind = (int)nx();
      rp->nk_seen = nx();
      const int64_t nko = nx();
      if (nko < 0 || nko > rp->max_keys) throw Error(SDH_E_INVALID, "bad snapshot key order");
      rp->korder_kid.resize((size_t)nko);
      rp->korder_key.resize((size_t)nko);
      for (int64_t j = 0; j < nko; ++j) {
        rp->korder_kid[(size_t)j] = nx();
        rp->korder_key[(size_t)j] = nx();
      }
      rp->fan.clear();
    }
    if ((size_t)nx() != e->psets.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    for (auto& pp : e->psets) {
      auto& ps = *pp;
      if (nx() != ps.partition || nx() != ps.kind) throw Error(SDH_E_INVALID, "snapshot of a different program");
      const int64_t cap = nx(), key_cap = nx();
      if (cap < 1 || cap > (1 << 20) || key_cap < 0 || key_cap > (int64_t)1 << 40)
        throw Error(SDH_E_INVALID, "bad snapshot K_part table size");
      ps.cap = (int)cap;
      ps.key_cap = 0;
      ps.st.n = 0;  // reallocated at the snapshot's capacity
      if (ps.st.p) HIPCHK(hipFree(ps.st.p));
      ps.st.p = nullptr;
      part_grow(e, ps, key_cap);
      if (ps.key_cap != key_cap) throw Error(SDH_E_INVALID, "snapshot key capacity mismatch");
      get_dev(ps.st.p, (size_t)2 * ps.key_cap * ps.n_groups * ps.bw() * 64 * 8);
      get_dev(ps.cur.p, (size_t)ps.key_cap * 4);
    }
    if ((size_t)nx() != e->seq_tail.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    for (size_t st = 0; st < e->seq_tail.size(); ++st) {
      const int64_t tl = nx();
      if (tl < 0 || tl > SEQ_TMAX) throw Error(SDH_E_INVALID, "bad snapshot tail length");
      e->seq_tail_len[st] = (int32_t)tl;
      get_dev(e->seq_tail[st].p, SEQ_TMAX * SEQ_TW * 8);
    }
    if ((size_t)nx() != e->ssets.size()) throw Error(SDH_E_INVALID, "snapshot of a different program");
    for (auto& up : e->ssets) {
      auto& ss = *up;
      if (nx() != ss.partition) throw Error(SDH_E_INVALID, "snapshot of a different program");
      const int64_t key_cap = nx(), ng = nx(), lds = nx(), words = nx();
      if (ng != ss.n_groups || key_cap < 0 || key_cap > ((int64_t)1 << 32) || words < 0 || lds < 64 || lds > 13312)
        throw Error(SDH_E_INVALID, "bad snapshot K_slab set");
      ss.lds_words = (int)lds;
      ss.key_cap = 0;
      ss.dir.n = 0;
      if (ss.dir.p) HIPCHK(hipFree(ss.dir.p));
      ss.dir.p = nullptr;
      slab_grow_keys(e, ss, key_cap);
      if (ss.key_cap != key_cap) throw Error(SDH_E_INVALID, "snapshot key capacity mismatch");
      get_dev(ss.dir.p, (size_t)key_cap * ng * 8);
      DevBuf<uint32_t> packed;
      packed.ensure(std::max<int64_t>(1, words));
      get_dev(packed.p, (size_t)words * 4);
      slab_init(e, ss, std::max<int64_t>(1 << 16, 2 * (words / ss.nsub) + 65536));
      get_dev(ss.live.p, 256 * 8);
      DevBuf<unsigned long long> zt;
      DevBuf<uint32_t*> pr;
      DevBuf<int64_t> pc;
      zt.ensure(1);
      pr.ensure(1);
      pc.ensure(1);
      const int64_t pcap = std::max<int64_t>(4, words);
      HIPCHK(hipMemset(zt.p, 0, 8));
      HIPCHK(hipMemcpy(pr.p, &packed.p, sizeof(uint32_t*), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(pc.p, &pcap, 8, hipMemcpyHostToDevice));
      if (words && !slab_move_raw(e, ss, ss.dir.p, pr.p, pc.p, zt.p, 1, std::vector<unsigned long long>(1, ~0ull), {},
                                  ss.d_ring.p, ss.d_cap.p, ss.head.p, ss.tail.p, ss.nsub))
        throw Error(SDH_E_CAPACITY, "K_slab restore: a ring overflowed");
      slab_heads(e, ss);
      ss.h_push0 = ss.h_head;
    }
    e->g_dev_matches = 0;
    e->device_matches = 0;
    e->r_matches = 0;
    e->r_blocks_used = 0;
    table_clear(e);
    e->broken.clear();
    return SDH_OK;
  });
}

void sdh_free(void* p) { free(p); }

void sdh_engine_destroy(sdh_engine* e) {
  if (!e) return;
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  if (e->h2d) (void)hipStreamSynchronize(e->h2d);
  for (hipEvent_t ev : {e->ev_h0, e->ev_h1, e->ev_stage[0], e->ev_stage[1]})
    if (ev) (void)hipEventDestroy(ev);
  if (e->h2d) (void)hipStreamDestroy(e->h2d);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

const char* sdh_last_error(sdh_engine* e) { return e ? e->err.c_str() : g_create_error.c_str(); }

}  // extern "C"

// knobs.h (t_knobs: the engine whose ABI call runs on this thread)
const char* sdh::knob(const char* name) {
  if (!t_knobs) return nullptr;
  for (const auto& kv : *t_knobs)
    if (kv.first == name) return kv.second.c_str();
  return nullptr;
}
