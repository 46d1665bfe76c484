// gen_lower.h -- host-side lowering of the pattern IR (siddhi_amd/ir.py) to K_gen device programs.
//
// Restates what StateInputStreamParser (core/util/parser/StateInputStreamParser.java:77-398) fixes at
// build time and the reference then walks at run time: the per-state links, the receivers' processor
// registration order, and the init / reset / update traversal orders of the inner-state-runtime tree
// (state/runtime/{Stream,Next,Every,Logical,Count}InnerStateRuntime.java), flattened into arrays so
// that the device never recurses.
#pragma once
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "kgen.h"

namespace sdh {
namespace kg {

struct LInsn {
  int op, lt, rt, res;
  int64_t a, b, imm;
};
using LCode = std::vector<LInsn>;
struct LState {
  int kind, stream, is_start, min, max, ltype, partner, next_pre, next_every, within_every, callback, this_last,
      has_selector;
  int64_t waiting;  // K_ABSENT: the 'for' time (ms), else -1
  std::vector<LCode> filters;
};
struct LRecv {
  int stream, kind;
  std::vector<int> procs;
};
struct LNode {
  int type, a, b, pre;
};
struct LQuery {
  int type, partition;
  int64_t within;
  std::vector<LState> st;
  std::vector<int> start_ids;
  std::vector<LRecv> recvs;
  std::vector<LNode> nodes;
};
struct LPartKey {
  int stream;
  LCode code;
};
struct LFanOut {  // a stream the partition's queries read but no key covers (every key sees it)
  int stream;
  int32_t id_hash;  // String.hashCode of the stream id
  int id_len;
};
struct LPart {
  std::vector<LPartKey> keys;
  std::vector<int> queries;
  std::vector<LFanOut> fanout;
  const LFanOut* fan(int stream) const {
    for (const auto& f : fanout)
      if (f.stream == stream) return &f;
    return nullptr;
  }
};
struct LProgram {
  std::vector<std::vector<int>> stream_types;
  std::vector<LQuery> q;
  std::vector<LPart> parts;
};

struct LowerError : std::runtime_error {
  explicit LowerError(const std::string& m) : std::runtime_error(m) {}
};

inline LProgram read_program(const void* blob, size_t len) {
  if (!blob || len < 16 || std::memcmp(blob, "SDHIR001", 8) != 0) throw LowerError("bad IR magic");
  const int64_t* w = reinterpret_cast<const int64_t*>(static_cast<const char*>(blob) + 8);
  const size_t n = (len - 8) / 8;
  size_t i = 0;
  auto nx = [&]() -> int64_t {
    if (i >= n) throw LowerError("IR blob truncated");
    return w[i++];
  };
  auto code = [&]() {
    LCode c((size_t)nx());
    for (auto& x : c) {
      const int64_t w0 = nx();
      x.op = (int)(w0 & 0xff);
      x.lt = (int)((w0 >> 8) & 0xff);
      x.rt = (int)((w0 >> 16) & 0xff);
      x.res = (int)((w0 >> 24) & 0xff);
      x.a = nx();
      x.b = nx();
      x.imm = nx();
    }
    return c;
  };
  LProgram p;
  if (nx() != 2) throw LowerError("unsupported IR version");
  p.stream_types.resize((size_t)nx());
  for (auto& s : p.stream_types) {
    s.resize((size_t)nx());
    for (auto& t : s) t = (int)nx();
  }
  const int64_t ns = nx();
  for (int64_t k = 0; k < ns; ++k) {
    const int64_t nb = nx();
    for (int64_t j = 0; j < (nb + 7) / 8; ++j) nx();
  }
  p.q.resize((size_t)nx());
  for (auto& q : p.q) {
    q.type = (int)nx();
    q.within = nx();
    q.st.resize((size_t)nx());
    q.partition = (int)nx();
    nx();
    for (auto& s : q.st) {
      s.kind = (int)nx(); s.stream = (int)nx(); s.is_start = (int)nx();
      s.min = (int)nx(); s.max = (int)nx(); s.ltype = (int)nx();
      s.partner = (int)nx(); s.next_pre = (int)nx(); s.next_every = (int)nx();
      s.within_every = (int)nx(); s.callback = (int)nx(); s.this_last = (int)nx();
      s.has_selector = (int)nx();
      s.waiting = nx();
      s.filters.resize((size_t)nx());
      for (auto& f : s.filters) f = code();
    }
    q.start_ids.resize((size_t)nx());
    for (auto& x : q.start_ids) x = (int)nx();
    q.recvs.resize((size_t)nx());
    for (auto& r : q.recvs) {
      r.stream = (int)nx();
      r.kind = (int)nx();
      r.procs.resize((size_t)nx());
      for (auto& x : r.procs) x = (int)nx();
    }
    q.nodes.resize((size_t)nx());
    for (auto& d : q.nodes) {
      d.type = (int)nx(); d.a = (int)nx(); d.b = (int)nx(); d.pre = (int)nx();
    }
    const int64_t no = nx();
    for (int64_t k = 0; k < no; ++k) code();
  }
  p.parts.resize((size_t)nx());
  for (auto& pd : p.parts) {
    pd.keys.resize((size_t)nx());
    for (auto& k : pd.keys) {
      k.stream = (int)nx();
      k.code = code();
    }
    pd.queries.resize((size_t)nx());
    for (auto& x : pd.queries) x = (int)nx();
  }
  if (i < n)  // trailer: the partitions' fan-out streams
    for (auto& pd : p.parts) {
      pd.fanout.resize((size_t)nx());
      for (auto& f : pd.fanout) {
        f.stream = (int)nx();
        f.id_hash = (int32_t)nx();
        f.id_len = (int)nx();
      }
    }
  return p;
}

// a partition query that reads a fan-out stream (it runs on K_gen)
inline bool reads_fanout(const LProgram& P, int qi) {
  const int pi = P.q[qi].partition;
  if (pi < 0) return false;
  for (const auto& s : P.q[qi].st)
    if (P.parts[pi].fan(s.stream)) return true;
  return false;
}

enum { N_STREAM = 0, N_NEXT, N_EVERY, N_LOGICAL, N_COUNT };

// the inner-state-runtime recursions (oracle: Runtime::node_init/reset/update)
inline void tree_init(const LQuery& q, int n, std::vector<int>& out) {
  const LNode& d = q.nodes[n];
  switch (d.type) {
    case N_STREAM: case N_COUNT: out.push_back(d.pre); break;
    case N_NEXT: tree_init(q, d.a, out); tree_init(q, d.b, out); break;
    case N_EVERY: tree_init(q, d.a, out); break;
    case N_LOGICAL: tree_init(q, d.b, out); tree_init(q, d.a, out); break;
  }
}
inline void tree_reset(const LQuery& q, int n, std::vector<int>& out) {
  const LNode& d = q.nodes[n];
  switch (d.type) {
    case N_STREAM: case N_COUNT: case N_EVERY: out.push_back(d.pre); break;
    case N_NEXT: tree_reset(q, d.b, out); tree_reset(q, d.a, out); break;
    case N_LOGICAL: tree_reset(q, d.b, out); break;
  }
}
inline void tree_update(const LQuery& q, int n, std::vector<int>& out) {
  const LNode& d = q.nodes[n];
  switch (d.type) {
    case N_STREAM: case N_COUNT: case N_EVERY: out.push_back(d.pre); break;
    case N_NEXT: tree_update(q, d.a, out); tree_update(q, d.b, out); break;
    case N_LOGICAL: tree_update(q, d.b, out); break;
  }
}

struct Sizing {
  int R = 64, N = 128, LC = 48;  // StateEvents, event nodes, list capacity per instance
};

// Lower query qi; throws LowerError when the shape exceeds the device program limits.
inline GQuery lower_gen(const LProgram& P, int qi, const Sizing& sz) {
  const LQuery& q = P.q[qi];
  GQuery g;
  std::memset(&g, 0, sizeof g);
  const int S = (int)q.st.size();
  if (S < 1 || S > GMAXS) throw LowerError("too many states for the device program");
  if (P.stream_types.size() > (size_t)GMAXSTREAM) throw LowerError("too many streams");
  g.qid = qi;
  g.type = q.type;
  g.n_states = S;
  g.partition = q.partition;
  g.within = q.within;
  g.n_start = (int)q.start_ids.size();
  if (g.n_start > GMAXS) throw LowerError("too many start states");
  for (int k = 0; k < g.n_start; ++k) g.start_ids[k] = q.start_ids[k];
  for (const auto& r : q.recvs) {
    if (r.stream < 0 || r.stream >= GMAXSTREAM || r.procs.size() > (size_t)GMAXS) throw LowerError("receiver");
    g.recv_kind[r.stream] = r.kind;
    g.recv_n[r.stream] = (int)r.procs.size();
    for (size_t k = 0; k < r.procs.size(); ++k) g.recv_procs[r.stream][k] = r.procs[k];
  }
  std::vector<int> o;
  if (!q.nodes.empty()) tree_init(q, 0, o);
  if (o.size() > (size_t)GMAXS) throw LowerError("runtime tree");
  g.n_init = (int)o.size();
  for (size_t k = 0; k < o.size(); ++k) g.init_order[k] = o[k];
  o.clear();
  if (!q.nodes.empty()) tree_reset(q, 0, o);
  if (o.size() > (size_t)(2 * GMAXS)) throw LowerError("runtime tree");
  g.n_reset = (int)o.size();
  for (size_t k = 0; k < o.size(); ++k) g.reset_order[k] = o[k];
  o.clear();
  if (!q.nodes.empty()) tree_update(q, 0, o);
  if (o.size() > (size_t)(2 * GMAXS)) throw LowerError("runtime tree");
  g.n_update = (int)o.size();
  for (size_t k = 0; k < o.size(); ++k) g.update_order[k] = o[k];

  // node attribute words: per stream, the attributes any filter reads through a slot
  std::vector<std::vector<int>> caps(P.stream_types.size());
  for (const auto& s : q.st)
    for (const auto& f : s.filters)
      for (const auto& in : f)
        if (in.op == OP_ATTR) {
          if (in.a < 0 || in.a >= S) throw LowerError("bad slot");
          const int stream = q.st[in.a].stream;
          auto& v = caps[stream];
          if (std::find(v.begin(), v.end(), (int)in.imm) == v.end()) v.push_back((int)in.imm);
        }
  int NA = 1;
  for (size_t s = 0; s < caps.size(); ++s) {
    if (caps[s].size() > (size_t)GMAXNA) throw LowerError("too many referenced attributes");
    g.n_cap[s] = (int)caps[s].size();
    for (size_t j = 0; j < caps[s].size(); ++j) {
      g.cap_attr[s][j] = caps[s][j];
      g.cap_type[s][j] = P.stream_types[s][caps[s][j]];
    }
    NA = std::max<int>(NA, (int)caps[s].size());
  }
  // states and filter code
  int pc = 0;
  for (int i = 0; i < S; ++i) {
    const LState& s = q.st[i];
    GState& d = g.st[i];
    d.kind = s.kind; d.stream = s.stream; d.is_start = s.is_start; d.min = s.min; d.max = s.max;
    d.ltype = s.ltype; d.partner = s.partner; d.next_pre = s.next_pre; d.next_every = s.next_every;
    d.within_every = s.within_every; d.callback = s.callback; d.this_last = s.this_last;
    d.has_selector = s.has_selector;
    d.pad = 0;
    d.waiting = s.waiting;
    if (s.filters.size() > (size_t)GMAXF) throw LowerError("too many filters");
    d.n_filt = (int)s.filters.size();
    for (size_t f = 0; f < s.filters.size(); ++f) {
      d.fb[f] = pc;
      int depth = 0, maxd = 0;
      for (const auto& in : s.filters[f]) {
        if (pc >= GMAXCODE) throw LowerError("filter code too long");
        GInsn& x = g.code[pc++];
        x.op = (int8_t)in.op; x.lt = (int8_t)in.lt; x.rt = (int8_t)in.rt; x.res = (int8_t)in.res;
        x.a = (int32_t)in.a;
        x.b = in.b;
        x.imm = in.imm;
        if (in.op == OP_ATTR) {
          const auto& v = caps[q.st[in.a].stream];
          x.imm = std::find(v.begin(), v.end(), (int)in.imm) - v.begin();
        }
        switch (in.op) {
          case OP_CONST: case OP_ATTR: case OP_STREAM_IS_NULL: ++depth; break;
          case OP_CMP: case OP_AND: case OP_OR: case OP_ARITH: --depth; break;
          default: break;
        }
        maxd = std::max(maxd, depth);
      }
      if (maxd >= GSTACK) throw LowerError("filter expression too deep");
      d.fe[f] = pc;
    }
  }
  g.n_code = pc;
  g.max_depth = 0;
  for (int i = 0; i < g.n_states; ++i)
    for (int f = 0; f < g.st[i].n_filt; ++f)
      g.max_depth = std::max(g.max_depth, code_depth(g, g.st[i].fb[f], g.st[i].fe[f]));
  bool v32 = true;  // every captured attribute is 4 bytes or narrower
  for (int s = 0; s < (int)P.stream_types.size() && s < GMAXSTREAM; ++s)
    for (int j = 0; j < g.n_cap[s]; ++j)
      if (g.cap_type[s][j] == T_LONG || g.cap_type[s][j] == T_DOUBLE) v32 = false;
  bool absent = false;  // absent states' scheduler queues hold up to one list's worth of times
  for (int i = 0; i < S; ++i) absent |= q.st[i].kind == K_ABSENT || (q.st[i].kind == K_LOGICAL && q.st[i].waiting != -1);
  make_layout(g.lay, S, sz.R, sz.N, sz.LC, NA, v32, absent ? sz.LC : 0);
  lower_atoms_or_none(g);
  return g;
}

// Output order of the matches of one event across queries (R18): junction subscribers in
// definition order (a partition subscribes at its first query); inside a partition a key's junction
// holds the clones in the partition's query order -- the planner emits LPart::queries in
// PartitionRuntime.metaQueryRuntimeMap order -- and each clone's receiver emits at the end of its own
// chunk (oracle: deliver_to / run_chunk). Returns rank[q * n_streams + stream].
inline std::vector<int> output_ranks(const LProgram& P) {
  const int nq = (int)P.q.size(), ns = (int)P.stream_types.size();
  std::vector<int> rank((size_t)nq * ns, 0);
  for (int s = 0; s < ns; ++s) {
    std::vector<char> done(P.parts.size(), 0);
    int r = 0;
    for (int qi = 0; qi < nq; ++qi) {
      const int pi = P.q[qi].partition;
      if (pi < 0) {
        rank[(size_t)qi * ns + s] = r++;
        continue;
      }
      if (done[pi]) continue;
      done[pi] = 1;
      for (int pq : P.parts[pi].queries) rank[(size_t)pq * ns + s] = r++;
    }
  }
  return rank;
}

// partition key of an event: String.valueOf(value) identity on raw attribute words
// (ValuePartitionExecutor.java:34-40); NaN keys collapse to one canonical NaN
inline int64_t key_of_raw(int type, int64_t raw) {
  if (type == T_FLOAT) {
    uint32_t u = (uint32_t)raw;
    float f;
    std::memcpy(&f, &u, 4);
    return f != f ? 0x7fc00000 : (int64_t)u;
  }
  if (type == T_DOUBLE) {
    double d;
    std::memcpy(&d, &raw, 8);
    return d != d ? 0x7ff8000000000000LL : raw;
  }
  return raw;
}

}  // namespace kg
}  // namespace sdh
