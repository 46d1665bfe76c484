// slab_lower.h -- host side of K_slab (slab.h): which queries run on sparse per-partial entries,
// and their entry layout. Restates the structure StateInputStreamParser builds for the shapes of
// slab.h (core/util/parser/StateInputStreamParser.java:145-398): the chain of elements after e1
// (Next: current.last.next = next.first, :218-250; Logical: both sides share next / partners,
// :280-368; Count: ANY -> 0 / Integer.MAX_VALUE, :370-393), and which slots later filters read
// (ExpressionParser.java:1225-1380 variable positions).
#pragma once
#include <cstring>
#include <string>
#include <vector>

#include "gen_lower.h"
#include "slab.h"

namespace sdh {
namespace slab {

// Shape of query qi (lowered to g by kg::lower_gen), or false with *why set.
inline bool shape_of_query(const kg::LProgram& P, int qi, const kg::GQuery& g, Shape* out, std::string* why) {
  auto no = [&](const char* m) {
    if (why) *why = m;
    return false;
  };
  const kg::LQuery& q = P.q[qi];
  const int S = (int)q.st.size();
  if (q.type != kg::Q_PATTERN) return no("not a pattern");
  if (q.partition < 0) return no("unpartitioned");
  if (S < 2 || S > SL_MAXS) return no("state count");
  if (g.max_depth > kg::RSTACK) return no("filter too deep");
  if (q.within >= 0 && !(q.start_ids.size() == 1 && q.start_ids[0] == 0)) return no("within start ids");
  if (q.within < 0 && !q.start_ids.empty() && !(q.start_ids.size() == 1 && q.start_ids[0] == 0))
    return no("start ids");
  Shape sh;
  std::memset(&sh, 0, sizeof sh);
  sh.S = S;
  for (int k = 0; k < kg::GMAXSTREAM; ++k) sh.proc[k] = -1;
  for (int i = 0; i < SL_MAXS; ++i) {
    sh.elem[i] = -1;
    sh.partner[i] = -1;
    sh.cnt_ord[i] = -1;
    sh.nxt[i][0] = sh.nxt[i][1] = -1;
    sh.drop[i][0] = sh.drop[i][1] = -1;
    sh.o_seq[i] = sh.o_cf[i] = sh.o_cl[i] = -1;
  }
  for (int i = 0; i < S; ++i) {
    const kg::LState& s = q.st[i];
    if (s.kind == kg::K_ABSENT || s.waiting != -1) return no("absent state");
    if (s.callback != -1 || s.within_every != -1) return no("callback / within-every");
    if (i > 0 && (s.is_start || s.next_every != -1 || s.this_last != i)) return no("inner every / start");
    if (s.stream < 0 || s.stream >= kg::GMAXSTREAM) return no("stream");
    if (sh.proc[s.stream] != -1) return no("two states read one stream");
    sh.proc[s.stream] = i;
    sh.kind[i] = s.kind;
    sh.ltype[i] = s.ltype;
    sh.min[i] = s.min;
    sh.max[i] = s.max;
    sh.has_sel[i] = s.has_selector;
    sh.partner[i] = s.kind == kg::K_LOGICAL ? s.partner : -1;
  }
  const kg::LState& e1 = q.st[0];
  if (e1.kind != kg::K_STREAM || !e1.is_start || e1.has_selector) return no("start state");
  if (e1.next_every != 0 && e1.next_every != -1) return no("every scope");
  sh.every = e1.next_every == 0;
  // receivers: one processor per stream (PatternSingleProcessStreamReceiver)
  for (const auto& r : q.recvs)
    if (r.procs.size() != 1 || q.st[r.procs[0]].stream != r.stream) return no("receiver");
  for (int i = 0; i < S; ++i) {
    bool found = false;
    for (const auto& r : q.recvs) found |= r.procs[0] == i;
    if (!found) return no("state without receiver");
  }
  // chain elements
  std::vector<std::vector<int>> el;
  el.push_back({0});
  sh.elem[0] = 0;
  int cur = e1.next_pre, n_count = 0;
  while (cur >= 0) {
    if (cur >= S || sh.elem[cur] != -1) return no("chain");
    const kg::LState& s = q.st[cur];
    std::vector<int> ids{cur};
    if (s.kind == kg::K_LOGICAL) {
      const int p = s.partner;
      if (p < 0 || p >= S || sh.elem[p] != -1 || q.st[p].kind != kg::K_LOGICAL || q.st[p].partner != cur ||
          q.st[p].ltype != s.ltype || q.st[p].next_pre != s.next_pre || q.st[p].has_selector != s.has_selector)
        return no("logical pair");
      ids.push_back(p);
    } else if (s.kind == kg::K_COUNT) {
      if (s.min < 1 || s.max > SL_CMAX || s.min > s.max) return no("count bounds");
      if (el.back().size() == 1 && q.st[el.back()[0]].kind == kg::K_COUNT) return no("two counts in a row");
      if (n_count >= SL_MAXCOUNT) return no("count states");
      sh.cnt_ord[cur] = n_count++;
    } else if (s.kind != kg::K_STREAM) {
      return no("state kind");
    }
    const int e = (int)el.size();
    for (int x : ids) sh.elem[x] = e;
    el.push_back(ids);
    cur = s.next_pre;
  }
  for (int i = 0; i < S; ++i)
    if (sh.elem[i] < 0) return no("state outside the chain");
  sh.n_elem = (int)el.size();
  for (size_t e = 0; e < el.size(); ++e) {
    const bool last = e + 1 == el.size();
    for (int x : el[e]) {
      if ((bool)q.st[x].has_selector != (last && e > 0)) return no("selector position");
      if (!last)
        for (size_t k = 0; k < el[e + 1].size(); ++k) sh.nxt[x][k] = el[e + 1][k];
    }
  }
  // count states drop a partial once slot id+1 or id+2 is filled (CountPreStateProcessor:60-66)
  for (int i = 0; i < S; ++i)
    if (sh.kind[i] == kg::K_COUNT) {
      sh.drop[i][0] = i + 1 < S ? i + 1 : -1;
      sh.drop[i][1] = i + 2 < S ? i + 2 : -1;
    }
  // which copies of which slots are read: another state's filter reads slot a (count: [0] -> first,
  // [last] -> last copy); a count's own filter reads its chain's first ([0] once it is not the
  // appended event) and previous ([last] unshifted = -2) events from copies
  std::vector<char> need_f(S, 0), need_l(S, 0);
  for (int st = 0; st < S; ++st)
    for (int f = 0; f < g.st[st].n_filt; ++f)
      for (int pc = g.st[st].fb[f]; pc < g.st[st].fe[f]; ++pc) {
        const kg::GInsn& in = g.code[pc];
        if (in.op != kg::OP_ATTR && in.op != kg::OP_STREAM_IS_NULL) continue;
        const int a = in.a;
        const int64_t b = in.b;
        if (a < 0 || a >= S) return no("slot");
        if (a == st) {
          if (sh.kind[st] == kg::K_COUNT) {
            if (b == 0) need_f[a] = 1;
            else if (b == -2) need_l[a] = 1;
            else if (b != -1) return no("count index");
          }
          continue;  // (one-event slots: other indexes read null)
        }
        if (sh.kind[a] == kg::K_COUNT) {
          if (b == 0) need_f[a] = 1;
          else if (b == -1) need_l[a] = 1;
          else return no("count index");
        } else if (b == 0 || b == -1) {
          need_f[a] = 1;
        }
      }
  // words: header, then sequence numbers, then captured copies
  int o = SL_HDR, nb = 0;
  for (int i = 0; i < S; ++i) {
    const bool last = sh.elem[i] == sh.n_elem - 1;
    bool store = i == 0 || sh.kind[i] == kg::K_COUNT || !last;
    if (sh.kind[i] == kg::K_LOGICAL && sh.ltype[i] == kg::L_AND) store = true;  // a side fills first
    if (store) {
      sh.o_seq[i] = o;
      o += 2 * (sh.kind[i] == kg::K_COUNT ? sh.max[i] : 1);
    }
  }
  for (int i = 0; i < S; ++i) {
    const int s = q.st[i].stream;
    sh.ncap[i] = g.n_cap[s];
    for (int j = 0; j < g.n_cap[s]; ++j)
      if (g.cap_type[s][j] == kg::T_LONG || g.cap_type[s][j] == kg::T_DOUBLE) {
        if (need_f[i] || need_l[i]) return no("8-byte captured attribute");
      }
    if (need_f[i]) {
      sh.o_cf[i] = o;
      o += sh.ncap[i];
      sh.nb_f[i] = nb;
      nb += sh.ncap[i];
    }
    if (need_l[i]) {
      sh.o_cl[i] = o;
      o += sh.ncap[i];
      sh.nb_l[i] = nb;
      nb += sh.ncap[i];
    }
  }
  if (nb > 32) return no("captured words");
  if (o > SL_MAXEW) return no("entry words");
  sh.EW = o;
  int n_const = 0;
  kg::const_ranks(g, sh.crank, &n_const);
  *out = sh;
  return true;
}

}  // namespace slab
}  // namespace sdh
