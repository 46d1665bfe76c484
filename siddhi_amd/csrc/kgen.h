// kgen.h -- K_gen: the general NFA interpreter, one lane per query instance (query, partition key).
//
// Restates the reference's object model for ONE state-stream runtime, so every query shape the IR
// expresses runs on the device: stream / count `<n:m>` / logical and-or states, PATTERN and
// SEQUENCE semantics, every scopes, `within` and within-every re-arming, count callbacks
// (startStateReset), partitions (one instance per key). Paths relative to siddhi-core
// .../query/input/stream/state/ (= state/):
//
//   objects     StateEvent (slots of StreamEvent chains; event/state/StateEvent.java:42-258),
//               shallow every-clones (event/state/StateEventCloner.java:46-58), StreamEvent
//               copies with their own `next` link; a per-instance pool of each, reclaimed by
//               mark/sweep from the pending / newAndEvery lists (the JVM's job in the reference)
//   lists       pending + newAndEvery per pre-processor, two-phase promotion
//               (StreamPreStateProcessor.java:203-227,281-289)
//   processors  StreamPre.processAndReturn:292-337, CountPre:53-156, LogicalPre:57-183,
//               StreamPost:53-72, CountPost:45-95, LogicalPost:59-87
//   runtime     init / reset / update orders of the inner-state-runtime tree (state/runtime/*),
//               flattened on the host; receivers (PatternMultiProcessStreamReceiver.java:38-44)
//
// The code is written once for host and device (KG_FN): the device kernel (nfa_gen.hip) runs it
// per lane over lane-interleaved arenas in HBM; tests/native builds the same header for the host
// to cross-check the restatement against the oracle (test infrastructure only).
#pragma once
#ifndef __HIPCC_RTC__  // (hiprtc: spec.hip supplies the fixed-width types)
#include <math.h>
#include <stdint.h>
#endif

#ifdef __HIPCC__
#define KG_FN __host__ __device__ inline
#define KG_UNROLL _Pragma("unroll")
#else
#define KG_FN inline
#define KG_UNROLL _Pragma("GCC unroll 8")
#endif

namespace sdh {
namespace kg {

constexpr int GMAXS = 8;         // states per query
constexpr int GMAXF = 4;         // filters per state
constexpr int GMAXCODE = 192;    // bytecode instructions per query
constexpr int GMAXNA = 8;        // captured attributes per node (per stream)
constexpr int GMAXSTREAM = 8;    // streams a query may read
constexpr int GSTACK = 12;       // bytecode evaluation stack
constexpr int GMAXNU = 4;        // node used-bitmask words the LDS hot cache holds (small pools)
constexpr int GMAXPOOL = 4096;   // StateEvents / nodes per instance after growth (record <= ring margin)
// the current event, not yet copied into the node pool: a stream / logical state's slot holds it
// while that state's filters run, and it is copied only when they pass (fewer pool writes and
// sweeps; observable behaviour is unchanged, the copy is invisible until a post processor runs)
constexpr int VNODE = 0x7fff;

enum { T_INT = 0, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_STRING };
enum { OP_CONST = 1, OP_ATTR, OP_IS_NULL, OP_STREAM_IS_NULL, OP_CMP, OP_AND, OP_OR, OP_NOT, OP_ARITH };
enum { CMP_EQ = 0, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE };
enum { AR_ADD = 0, AR_SUB, AR_MUL, AR_DIV, AR_MOD };
enum { K_STREAM = 0, K_COUNT, K_LOGICAL, K_ABSENT };  // K_ABSENT: AbsentStreamPre/PostStateProcessor
enum { L_AND = 0, L_OR };
enum { Q_PATTERN = 0, Q_SEQUENCE };
enum { R_SINGLE = 0, R_MULTI };

// error codes (per lane, first one wins)
enum { GE_OK = 0, GE_CAPACITY = 1, GE_REFERENCE = 2 };
// capacity kinds: the pools and lists grow (the engine re-lays the arenas and re-runs the push);
// CAP_FIXED: the GC pin stack depth (4) is compiled in
enum { CAP_STATES = 1, CAP_NODES = 2, CAP_LIST = 4, CAP_FIXED = 8 };

struct GInsn {
  int8_t op, lt, rt, res;
  int32_t a;     // slot (state id) for ATTR / STREAM_IS_NULL
  int64_t b;     // chain index (CURRENT=-1, LAST=-2, ...)
  int64_t imm;   // constant bits / node attribute word / cmp or arith op
};

struct GState {
  int32_t kind, stream, is_start, min, max, ltype, partner, next_pre, next_every, within_every, callback,
      this_last, has_selector;
  int32_t n_filt;
  int32_t fb[GMAXF], fe[GMAXF];   // filter code ranges
  int32_t pad;
  int64_t waiting;                // K_ABSENT: the 'for' time (ms)
};

// arena layout (word offsets; 32-bit and 64-bit arenas, lane-interleaved on the device)
struct GLayout {
  int32_t S, R, N, LC, NA, NU;     // states, StateEvents, nodes, list capacity, node attrs, node-mask words
  int32_t o_flags, o_pn, o_nn, o_plist, o_nlist, o_seslot, o_ndnext, o_ndnull, o_init, n32;
  int32_t o_seused, o_ndused, o_sets, o_ndseq, o_ndts, o_ndval, n64;
  int32_t v32;  // node attribute words in the 32-bit arena (every captured type is 4 bytes or less)
  // pools beyond the LDS hot cache (R > 64 StateEvents or N > 64 * GMAXNU nodes): the used-bitmasks
  // stay in the arena (SU / NU words) and mark/sweep marks into o_mark (SU + NU words, 64-bit arena)
  int32_t SU, big, o_mark, pad;
  // absent states' schedulers (TQ > 0 only for queries with absent states): per state a FIFO ring of
  // notification times o_tq [state][TQ] and lastScheduledTime o_lst (64-bit arena), ring head /
  // length o_tqh [state][2] (32-bit arena)
  int32_t TQ, o_tq, o_lst, o_tqh;
  int32_t o_ret, pad2;  // the partials one processAndReturn / timer returns (LC entries: they grow with the lists)
};

// K_seq compare atoms: a state's filters as a conjunction of typed compares whose operands are a
// leaf (a slot's attribute word or a bytecode constant) or one arithmetic op over two leaves -- the
// same Java semantics as eval_code, without the evaluation stack (kg::lower_atoms, seq_match)
constexpr int GMAXATOM = 16;
// LF_ATTR0: a slot reference with chain index 0 (the chain's first event; in a one-event window
// slot the same event as LF_ATTR's CURRENT / 0)
enum { LF_ATTR = 0, LF_CONST = 1, LF_NULL = 2, LF_ATTR0 = 3 };
constexpr int GMAXCONST = 16;  // CONST leaves of one query's atoms
struct GLeaf {
  int8_t kind, slot, cap, type;
  int16_t pc;     // LF_CONST: instruction whose imm is the (per-lane) constant
  int16_t cslot;  // LF_CONST: index into GQuery::const_pc (staged per lane on the device)
};
struct GOpnd {
  GLeaf a, b;
  int8_t arith;  // -1: leaf a alone; else AR_* over (a, b) with operand types a.type / b.type
  int8_t res;
  int8_t pad[6];
};
struct GAtom {
  int8_t state, op, lt, rt;
  int32_t pad;
  GOpnd l, r;
};

struct GQuery {
  int32_t qid, type, n_states, partition, rank;
  int32_t pad0;
  int64_t within;                                  // ms, -1 = none
  int32_t n_start, start_ids[GMAXS];
  int32_t recv_kind[GMAXSTREAM], recv_n[GMAXSTREAM], recv_procs[GMAXSTREAM][GMAXS];
  int32_t n_init, init_order[GMAXS];               // node_init(0): init_pre order
  int32_t n_reset, reset_order[2 * GMAXS];         // node_reset(0): resetState order
  int32_t n_update, update_order[2 * GMAXS];       // node_update(0): updateState order
  int32_t n_cap[GMAXSTREAM], cap_attr[GMAXSTREAM][GMAXNA];  // node attribute words per stream
  int32_t cap_type[GMAXSTREAM][GMAXNA];
  GLayout lay;
  GState st[GMAXS];
  int32_t n_code;
  int32_t max_depth;  // deepest evaluation stack of any filter (kg::code_depth)
  GInsn code[GMAXCODE];
  int32_t n_atoms;    // > 0: every filter lowered to atoms (atom_begin[i] .. atom_begin[i+1] of state i)
  int32_t atom_begin[GMAXS + 1];
  GAtom atoms[GMAXATOM];
  int32_t n_const;    // CONST leaves of the atoms: their instructions
  int32_t const_pc[GMAXCONST];
};

// ---- Java value semantics (executor/condition/compare/**, executor/math/**) ----
struct Val {
  int32_t type;
  int32_t null;
  int64_t bits;   // int/long/bool/string id (sign-extended), float bits (low 32), double bits
};

KG_FN float f_of(int64_t b) { union { uint32_t u; float f; } x; x.u = (uint32_t)b; return x.f; }
KG_FN double d_of(int64_t b) { union { int64_t i; double d; } x; x.i = b; return x.d; }
KG_FN int64_t bits_f(float f) { union { uint32_t u; float f; } x; x.f = f; return (int64_t)x.u; }
KG_FN int64_t bits_d(double d) { union { int64_t i; double d; } x; x.d = d; return x.i; }

KG_FN float as_f(const Val& v) {
  switch (v.type) {
    case T_INT: return (float)(int32_t)v.bits;
    case T_LONG: return (float)v.bits;
    case T_FLOAT: return f_of(v.bits);
    default: return (float)d_of(v.bits);
  }
}
KG_FN double as_d(const Val& v) {
  switch (v.type) {
    case T_INT: return (double)(int32_t)v.bits;
    case T_LONG: return (double)v.bits;
    case T_FLOAT: return (double)f_of(v.bits);
    default: return d_of(v.bits);
  }
}

template <class T>
KG_FN bool cmp_op(int op, T a, T b) {
  switch (op) {
    case CMP_EQ: return a == b;
    case CMP_NE: return a != b;
    case CMP_GT: return a > b;
    case CMP_GE: return a >= b;
    case CMP_LT: return a < b;
    default: return a <= b;
  }
}

// the typed compare table (compare/*/...Executor*.java execute() at :33-38)
KG_FN bool typed_compare(int op, const Val& l, const Val& r) {
  const int lt = l.type, rt = r.type;
  if (lt == T_STRING || lt == T_BOOL) {
    const bool eq = l.bits == r.bits;
    return op == CMP_EQ ? eq : !eq;
  }
  const bool is_eq = (op == CMP_EQ || op == CMP_NE);
  if (lt == T_DOUBLE || rt == T_DOUBLE) return cmp_op(op, as_d(l), as_d(r));
  if (lt == T_FLOAT || rt == T_FLOAT) {
    if (is_eq && (lt == T_LONG || rt == T_LONG)) return cmp_op(op, as_d(l), as_d(r));  // ...LongFloat.java:36
    return cmp_op(op, as_f(l), as_f(r));
  }
  if (lt == T_LONG || rt == T_LONG) return cmp_op(op, l.bits, r.bits);
  return cmp_op(op, (int32_t)l.bits, (int32_t)r.bits);
}

// executor/math/{add,subtract,multiply,divide,mod}: null in -> null; /0 and %0 -> null for every
// type (0.0f / -0.0 included, DivideExpressionExecutorFloat.java:46); integer ops wrap
KG_FN Val arith(int op, int res, const Val& l, const Val& r) {
  Val v{res, 1, 0};
  if (l.null || r.null) return v;
  v.null = 0;
  if (res == T_INT) {
    const int32_t a = (int32_t)l.bits, b = (int32_t)r.bits;
    const uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
    switch (op) {
      case AR_ADD: v.bits = (int32_t)(ua + ub); break;
      case AR_SUB: v.bits = (int32_t)(ua - ub); break;
      case AR_MUL: v.bits = (int32_t)(ua * ub); break;
      case AR_DIV:
        if (b == 0) { v.null = 1; return v; }
        v.bits = (a == INT32_MIN && b == -1) ? INT32_MIN : a / b;
        break;
      default:
        if (b == 0) { v.null = 1; return v; }
        v.bits = (b == -1) ? 0 : a % b;
    }
  } else if (res == T_LONG) {
    const int64_t a = l.bits, b = r.bits;
    const uint64_t ua = (uint64_t)a, ub = (uint64_t)b;
    switch (op) {
      case AR_ADD: v.bits = (int64_t)(ua + ub); break;
      case AR_SUB: v.bits = (int64_t)(ua - ub); break;
      case AR_MUL: v.bits = (int64_t)(ua * ub); break;
      case AR_DIV:
        if (b == 0) { v.null = 1; return v; }
        v.bits = (a == INT64_MIN && b == -1) ? INT64_MIN : a / b;
        break;
      default:
        if (b == 0) { v.null = 1; return v; }
        v.bits = (b == -1) ? 0 : a % b;
    }
  } else if (res == T_FLOAT) {
    const float a = as_f(l), b = as_f(r);
    float o;
    switch (op) {
      case AR_ADD: o = a + b; break;
      case AR_SUB: o = a - b; break;
      case AR_MUL: o = a * b; break;
      case AR_DIV: if (b == 0.0f) { v.null = 1; return v; } o = a / b; break;
      default: if (b == 0.0f) { v.null = 1; return v; } o = fmodf(a, b);
    }
    v.bits = bits_f(o);
  } else {
    const double a = as_d(l), b = as_d(r);
    double o;
    switch (op) {
      case AR_ADD: o = a + b; break;
      case AR_SUB: o = a - b; break;
      case AR_MUL: o = a * b; break;
      case AR_DIV: if (b == 0.0) { v.null = 1; return v; } o = a / b; break;
      default: if (b == 0.0) { v.null = 1; return v; } o = fmod(a, b);
    }
    v.bits = bits_d(o);
  }
  return v;
}

// Shape-compiled filters (spec.hip generates straight-line code from a shape's bytecode): one
// helper per instruction kind, the instruction's static fields as template arguments, so every
// type / operator dispatch of eval_code folds away at compile time. Same semantics, instruction
// by instruction, as eval_code above.
template <int RES>
KG_FN Val sp_const(int64_t imm) {
  return Val{RES, 0, RES == T_FLOAT ? (int64_t)(uint32_t)imm : RES == T_INT ? (int64_t)(int32_t)imm : imm};
}
template <int RES>
KG_FN Val sp_attr(int64_t raw, bool isnull) {
  Val x{RES, 1, 0};
  if (!isnull) {
    x.null = 0;
    x.bits = RES == T_INT ? (int64_t)(int32_t)raw : RES == T_FLOAT ? (int64_t)(uint32_t)raw : raw;
  }
  return x;
}
KG_FN Val sp_bool(bool b) { return Val{T_BOOL, 0, b ? 1 : 0}; }
KG_FN Val sp_is_null(const Val& x) { return sp_bool(x.null != 0); }
KG_FN Val sp_not(const Val& x) { return sp_bool(!(!x.null && x.bits)); }
KG_FN Val sp_and(const Val& l, const Val& r) { return sp_bool((!l.null && l.bits) && (!r.null && r.bits)); }
KG_FN Val sp_or(const Val& l, const Val& r) { return sp_bool((!l.null && l.bits) || (!r.null && r.bits)); }
template <int OP, int LT, int RT>
KG_FN Val sp_cmp(Val l, Val r) {
  l.type = LT;
  r.type = RT;
  return sp_bool(!l.null && !r.null && typed_compare(OP, l, r));
}
template <int OP, int RES, int LT, int RT>
KG_FN Val sp_arith(Val l, Val r) {
  l.type = LT;
  r.type = RT;
  return arith(OP, RES, l, r);
}
KG_FN bool sp_true(const Val& v) { return !v.null && v.bits; }

// ------------------------------------------------------------------------------------------
// per-lane runtime over the instance arena
// ------------------------------------------------------------------------------------------
enum { FL_CHANGED = 1, FL_INIT = 2, FL_SUCCESS = 4, FL_SSRESET = 8, FL_RETURNED = 16, FL_ITER = 32,
       FL_INACTIVE = 64 /* an absent start state without every that has fired (`active = false`) */ };

// The predicate bytecode's stack machine (ExpressionExecutor trees: executor/condition/**,
// executor/math/**, VariableExpressionExecutor.java:45-47). Structure comes from q (wave-uniform on
// the device), constants from the lane's own query ql. attr(in) resolves OP_ATTR to a typed value,
// stream_null(in) answers OP_STREAM_IS_NULL -- K_gen over its instance arena, K_seq over the
// event window of a sequence.
// Evaluation stacks. ArrStack: an indexed array (K_gen; private memory on the device). RegStack:
// a shift register of RSTACK entries, every access at a constant index, so it lives in VGPRs
// (K_seq, whose shapes are checked to need at most RSTACK entries, kg::code_depth).
struct ArrStack {
  Val st[GSTACK];
  int sp = 0;
  KG_FN void push(const Val& v) {
    st[sp++] = v;
    if (sp >= GSTACK) sp = GSTACK - 1;
  }
  KG_FN Val pop() { return st[--sp]; }
  KG_FN Val result() const { return sp == 1 ? st[0] : Val{T_BOOL, 1, 0}; }
};
constexpr int RSTACK = 6;
struct RegStack {
  Val s[RSTACK];
  int sp = 0;
  KG_FN void push(const Val& v) {
KG_UNROLL
    for (int k = RSTACK - 1; k > 0; --k) s[k] = s[k - 1];
    s[0] = v;
    ++sp;
  }
  KG_FN Val pop() {
    const Val v = s[0];
KG_UNROLL
    for (int k = 0; k < RSTACK - 1; ++k) s[k] = s[k + 1];
    --sp;
    return v;
  }
  KG_FN Val result() const { return sp == 1 ? s[0] : Val{T_BOOL, 1, 0}; }
};

// imm(pc): the lane's constant of CONST instruction pc (its own query's, or its column of a
// lane-interleaved constant table: kg::LaneConsts)
template <class Stack = ArrStack, class Imm, class Attr, class StreamNull>
KG_FN Val eval_code_imm(const GQuery* q, Imm imm_of, int b, int e, Attr attr, StreamNull stream_null) {
  Stack stk;
  for (int pc = b; pc < e; ++pc) {
    const GInsn& in = q->code[pc];
    switch (in.op) {
      case OP_CONST: {  // constants differ within a shape: the lane's own query
        const int64_t imm = imm_of(pc);
        Val v{in.res, 0, 0};
        if (in.res == T_FLOAT) v.bits = (int64_t)(uint32_t)imm;
        else if (in.res == T_INT) v.bits = (int32_t)imm;
        else v.bits = imm;
        stk.push(v);
        break;
      }
      case OP_ATTR:
        stk.push(attr(in));
        break;
      case OP_STREAM_IS_NULL:
        stk.push(Val{T_BOOL, 0, stream_null(in) ? 1 : 0});
        break;
      case OP_IS_NULL: {
        const Val x = stk.pop();
        stk.push(Val{T_BOOL, 0, x.null ? 1 : 0});
        break;
      }
      case OP_NOT: {  // NotConditionExpressionExecutor: only TRUE -> FALSE
        const Val x = stk.pop();
        stk.push(Val{T_BOOL, 0, (!x.null && x.bits) ? 0 : 1});
        break;
      }
      case OP_AND:
      case OP_OR: {
        const Val r = stk.pop();
        const Val l = stk.pop();
        const bool lb = !l.null && l.bits, rb = !r.null && r.bits;
        stk.push(Val{T_BOOL, 0, (in.op == OP_AND ? (lb && rb) : (lb || rb)) ? 1 : 0});
        break;
      }
      case OP_CMP: {  // CompareConditionExpressionExecutor.java:39-43
        // operand types are static (the planner's ltype/rtype): taking them from the instruction
        // keeps the typed dispatch wave-uniform
        Val r = stk.pop();
        Val l = stk.pop();
        l.type = in.lt;
        r.type = in.rt;
        stk.push(Val{T_BOOL, 0, (!l.null && !r.null && typed_compare((int)in.imm, l, r)) ? 1 : 0});
        break;
      }
      case OP_ARITH: {
        Val r = stk.pop();
        Val l = stk.pop();
        l.type = in.lt;
        r.type = in.rt;
        stk.push(arith((int)in.imm, in.res, l, r));
        break;
      }
      default:
        stk.push(Val{T_BOOL, 1, 0});
    }
  }
  return stk.result();
}

template <class Stack = ArrStack, class Attr, class StreamNull>
KG_FN Val eval_code(const GQuery* q, const GQuery* ql, int b, int e, Attr attr, StreamNull stream_null) {
  return eval_code_imm<Stack>(q, [&](int pc) { return ql->code[pc].imm; }, b, e, attr, stream_null);
}

// A lane's per-query values, read from the group's lane-interleaved constant table
// [group][slot][64] (engine.hip lane_consts): slot 0 the query id, 1 `within`, 2 + k the k-th CONST
// instruction of the shape in program order. A wave's 64 lanes read one slot as one coalesced 512-B
// row instead of 64 scattered lines of 64 different GQuery structs (K_slab and K_part read them per
// work item). col == nullptr: the lane's own query (host builds).
constexpr int LC_QID = 0, LC_WITHIN = 1, LC_FIRST = 2;
struct LaneConsts {
  const GQuery* ql;
  const int64_t* col;  // table + (group * slots) * 64 + lane
  KG_FN int64_t qid() const { return col ? col[LC_QID * 64] : (int64_t)ql->qid; }
  KG_FN int64_t within() const { return col ? col[LC_WITHIN * 64] : ql->within; }
  // k: the instruction's rank among the shape's CONST instructions
  KG_FN int64_t imm(int pc, int k) const { return col ? col[(LC_FIRST + k) * 64] : ql->code[pc].imm; }
};

#ifndef __HIPCC_RTC__
// per instruction its rank among the CONST instructions of the code (-1: not a CONST)
inline void const_ranks(const GQuery& g, int8_t* rank, int* n) {
  int k = 0;
  for (int pc = 0; pc < GMAXCODE; ++pc) rank[pc] = (pc < g.n_code && g.code[pc].op == OP_CONST) ? (int8_t)k++ : -1;
  *n = k;
}
#endif

struct Emitter;  // defined by the caller: void emit(const Ctx&, int se)
#ifdef KG_PROFILE
void kg_prof_hit(const GLayout& L, int is64, int off);
extern int g_prof_phase;  // census phase (0 = processing, 1 = mark/sweep)
#define KG_PHASE(p) (g_prof_phase = (p))
#else
#define KG_PHASE(p) ((void)0)
#endif

struct Ctx {
  // q: the query's structure. On the device it is the wave's template -- every lane of a group has
  // the same structure (the host groups queries by shape), so q is wave-uniform and its fields are
  // scalar loads. ql: the lane's own query, read only for what differs within a shape (bytecode
  // constants, `within`, qid). lay/within are cached in registers for the whole item.
  const GQuery* q;
  const GQuery* ql;
  GLayout lay;
  int64_t within;
  int32_t* w32;
  int64_t* w64;
  int64_t stride;
  // hot words, cached for the whole work item (LDS on the device, [word][lane]): per state flags /
  // pending count / newAndEvery count ([3][GMAXS]), and the two pools' used-bitmasks ([1 + GMAXNU]).
  // They are touched on every event by every processor (about half of all arena accesses on C3);
  // load_hot/store_hot move them between the arena and the cache at the item's ends.
  int32_t* h32;
  int64_t* h64;
  int64_t hstride;
  int32_t hs;  // states the h32 cache holds per field (the launch's max)
  // current event (the instance's view of it)
  int64_t seq, ts;
  int32_t stream;
  const int64_t* ev_val;  // [GMAXNA] the event's captured words (wave-uniform: LDS on the device)
  uint32_t ev_null;
  int32_t err;
  int32_t capk;  // GE_CAPACITY: CAP_* bits of the limits that were hit
  // The dynamically indexed arrays (event words, pins, return list) live outside Ctx, behind
  // pointers: an array indexed by a run-time value inside the struct would keep the whole Ctx in
  // scratch memory on the device (no SROA), turning every field read into a scratch load.
  // GC roots outside the lists: partials unlinked or not yet linked while they are worked on
  int32_t* pins;  // [4] (stride hstride: LDS on the device)
  int32_t npin;
  int32_t n_ret;  // partials returned so far (arena ret_at: GC roots until handed on)
  // the count state's chain as process_and_return just extended it (its last node and length), so
  // CountPost does not walk it again; -1 = unknown
  int32_t cnt_tail = -1;
  int64_t cnt_len = 0;
  // absent states: a timer is being processed (its matches are timer records, ordered by (timer_ts =
  // the running max of the times fired so far, query, partition key, emission order) before the
  // triggering event's own)
  bool in_timer = false;
  int64_t timer_ts = 0;

#ifdef KG_PROFILE  // host-only access census (tests/native, test infrastructure)
  int32_t& i32(int i) const { kg_prof_hit(lay, 0, i); return w32[(int64_t)i * stride]; }
  int64_t& i64(int i) const { kg_prof_hit(lay, 1, i); return w64[(int64_t)i * stride]; }
#else
  KG_FN int32_t& i32(int i) const { return w32[(int64_t)i * stride]; }
  KG_FN int64_t& i64(int i) const { return w64[(int64_t)i * stride]; }
#endif
  KG_FN const GState& S(int i) const { return q->st[i]; }
  KG_FN int nS() const { return lay.S; }
  // an absent side of a logical state (AbsentLogicalPre/PostStateProcessor); waiting -2 is a side
  // without 'for' (the reference's waitingTime -1)
  KG_FN bool absent_l(int i) const { return S(i).kind == K_LOGICAL && S(i).waiting != -1; }
  KG_FN int64_t wait_of(int i) const { return S(i).waiting == -2 ? -1 : S(i).waiting; }
  KG_FN bool absent_any(int i) const { return S(i).kind == K_ABSENT || absent_l(i); }
  KG_FN void bind(const GQuery* tmpl, const GQuery* own) {
    q = tmpl;
    ql = own;
    lay = tmpl->lay;
    within = own->within;
  }

  // ---- arena fields ----
  KG_FN int32_t& flags(int i) const { return h32[(int64_t)i * hstride]; }
  KG_FN int32_t& pn(int i) const { return h32[(int64_t)(hs + i) * hstride]; }
  KG_FN int32_t& nn(int i) const { return h32[(int64_t)(2 * hs + i) * hstride]; }
  KG_FN int32_t& pl(int i, int k) const { return i32(lay.o_plist + i * lay.LC + k); }
  KG_FN int32_t& nl(int i, int k) const { return i32(lay.o_nlist + i * lay.LC + k); }
  KG_FN int32_t& slot(int se, int i) const { return i32(lay.o_seslot + se * lay.S + i); }
  KG_FN int64_t& se_ts(int se) const { return i64(lay.o_sets + se); }
  KG_FN int32_t& nd_next(int n) const { return i32(lay.o_ndnext + n); }
  KG_FN int32_t& nd_null(int n) const { return i32(lay.o_ndnull + n); }
  KG_FN int64_t& nd_seq(int n) const { return i64(lay.o_ndseq + n); }
  KG_FN int64_t& nd_ts(int n) const { return i64(lay.o_ndts + n); }
  // node attribute words: raw words of 4-byte-or-narrower types are stored as their low 32 bits
  // and sign-extended back, which reproduces raw_word's value for every such column
  KG_FN int64_t nd_val(int n, int j) const {
    const int o = lay.o_ndval + n * lay.NA + j;
    return lay.v32 ? (int64_t)i32(o) : i64(o);
  }
  KG_FN void set_nd_val(int n, int j, int64_t v) const {
    const int o = lay.o_ndval + n * lay.NA + j;
    if (lay.v32) i32(o) = (int32_t)v;
    else i64(o) = v;
  }
  // absent states' schedulers: FIFO ring of notification times, its head / length, lastScheduledTime
  KG_FN int64_t& tq(int i, int k) const { return i64(lay.o_tq + i * lay.TQ + k); }
  KG_FN int32_t& tq_head(int i) const { return i32(lay.o_tqh + 2 * i); }
  KG_FN int32_t& tq_len(int i) const { return i32(lay.o_tqh + 2 * i + 1); }
  KG_FN int64_t& lst(int i) const { return i64(lay.o_lst + i); }
  KG_FN int32_t& ret_at(int k) const { return i32(lay.o_ret + k); }
  KG_FN void notify_at(int i, int64_t t) {  // Scheduler.notifyAt:118-126 (toNotifyQueue.put)
    const int n = tq_len(i);
    if (n >= lay.TQ) { cap_fail(CAP_LIST); return; }
    tq(i, (tq_head(i) + n) % lay.TQ) = t;
    tq_len(i) = n + 1;
  }
  // used-bitmask words: the LDS hot cache for small pools, the arena itself for big ones (lay.big is
  // the template's, so the choice is wave-uniform)
  KG_FN int64_t& se_used(int w) const { return lay.big ? i64(lay.o_seused + w) : h64[0]; }
  KG_FN int64_t& nd_used(int w) const { return lay.big ? i64(lay.o_ndused + w) : h64[(int64_t)(1 + w) * hstride]; }
  KG_FN void load_hot() {
    for (int i = 0; i < lay.S; ++i) {
      flags(i) = i32(lay.o_flags + i);
      pn(i) = i32(lay.o_pn + i);
      nn(i) = i32(lay.o_nn + i);
    }
    if (lay.big) return;
    h64[0] = i64(lay.o_seused);
    for (int w = 0; w < lay.NU; ++w) h64[(int64_t)(1 + w) * hstride] = i64(lay.o_ndused + w);
  }
  KG_FN void store_hot() const {
    for (int i = 0; i < lay.S; ++i) {
      i32(lay.o_flags + i) = flags(i);
      i32(lay.o_pn + i) = pn(i);
      i32(lay.o_nn + i) = nn(i);
    }
    if (lay.big) return;
    i64(lay.o_seused) = h64[0];
    for (int w = 0; w < lay.NU; ++w) i64(lay.o_ndused + w) = h64[(int64_t)(1 + w) * hstride];
  }

  KG_FN void fail(int e) {
    if (err == GE_OK) err = e;
  }
  KG_FN void cap_fail(int kind) {  // GE_CAPACITY, and which limit: the host grows it and re-runs
    capk |= kind;
    fail(GE_CAPACITY);
  }

  // ---- allocation with mark/sweep reclamation ----
  // mark bits: in registers for small pools, in the arena's o_mark words for big ones
  struct RegMarks {
    uint64_t s = 0, n[GMAXNU] = {0, 0, 0, 0};
    KG_FN bool se(int i) const { return (s >> i) & 1ull; }
    KG_FN void set_se(int i) { s |= 1ull << i; }
    KG_FN bool nd(int i) const { return (n[i >> 6] >> (i & 63)) & 1ull; }
    KG_FN void set_nd(int i) { n[i >> 6] |= 1ull << (i & 63); }
  };
  struct ArenaMarks {
    const Ctx* c;
    KG_FN int64_t& w(int k) const { return c->i64(c->lay.o_mark + k); }
    KG_FN bool se(int i) const { return ((uint64_t)w(i >> 6) >> (i & 63)) & 1ull; }
    KG_FN void set_se(int i) const { w(i >> 6) = (int64_t)((uint64_t)w(i >> 6) | (1ull << (i & 63))); }
    KG_FN bool nd(int i) const { return ((uint64_t)w(c->lay.SU + (i >> 6)) >> (i & 63)) & 1ull; }
    KG_FN void set_nd(int i) const {
      int64_t& x = w(c->lay.SU + (i >> 6));
      x = (int64_t)((uint64_t)x | (1ull << (i & 63)));
    }
  };
  template <class M>
  KG_FN void mark_chain(int n, M& m) const {
    while (n >= 0 && n < lay.N && !m.nd(n)) {
      m.set_nd(n);
      n = nd_next(n);
    }
  }
  template <class M>
  KG_FN void mark_se(int se, M& m) const {
    if (se < 0 || m.se(se)) return;
    m.set_se(se);
    for (int i = 0; i < nS(); ++i) mark_chain(slot(se, i), m);
  }
  template <class M>
  KG_FN void mark_roots(M& m) const {
    for (int i = 0; i < nS(); ++i) {
      for (int k = 0; k < pn(i); ++k) mark_se(pl(i, k), m);
      for (int k = 0; k < nn(i); ++k) mark_se(nl(i, k), m);
    }
    for (int k = 0; k < npin && k < 4; ++k) mark_se(pins[(int64_t)k * hstride], m);
    for (int k = 0; k < n_ret; ++k) mark_se(ret_at(k), m);
  }
  KG_FN void gc() {
    KG_PHASE(1);
    if (lay.big) {
      ArenaMarks m{this};
      for (int k = 0; k < lay.SU + lay.NU; ++k) m.w(k) = 0;
      mark_roots(m);
      for (int k = 0; k < lay.SU; ++k) se_used(k) = m.w(k);
      for (int k = 0; k < lay.NU; ++k) nd_used(k) = m.w(lay.SU + k);
    } else {
      RegMarks m;
      mark_roots(m);
      se_used(0) = (int64_t)m.s;
      for (int w = 0; w < lay.NU; ++w) nd_used(w) = (int64_t)m.n[w];
    }
    KG_PHASE(0);
  }
  KG_FN int find_free_se() const {
    for (int w = 0; w < lay.SU; ++w) {
      const int lim = lay.R - w * 64;
      const uint64_t u = (uint64_t)se_used(w);
      const uint64_t fr = ~u & (lim >= 64 ? ~0ull : ((1ull << lim) - 1));
      if (fr) return w * 64 + __builtin_ctzll(fr);
    }
    return -1;
  }
  KG_FN int find_free_nd() const {
    for (int w = 0; w < lay.NU; ++w) {
      const int lim = lay.N - w * 64;
      const uint64_t u = (uint64_t)nd_used(w);
      const uint64_t fr = ~u & (lim >= 64 ? ~0ull : ((1ull << lim) - 1));
      if (fr) return w * 64 + __builtin_ctzll(fr);
    }
    return -1;
  }
  KG_FN int new_state(bool blank = true) {  // blank = false: the caller writes every slot and ts
    int s = find_free_se();
    if (s < 0) {
      gc();
      s = find_free_se();
      if (s < 0) { cap_fail(CAP_STATES); return -1; }
    }
    se_used(s >> 6) = (int64_t)((uint64_t)se_used(s >> 6) | (1ull << (s & 63)));
    if (blank) {
      for (int i = 0; i < nS(); ++i) slot(s, i) = -1;
      se_ts(s) = -1;
    }
    return s;
  }
  KG_FN void pin(int se) {
    if (npin < 4) pins[(int64_t)npin * hstride] = se;
    else cap_fail(CAP_FIXED);  // an unrecorded root could be swept: refuse rather than risk it
    ++npin;
  }
  KG_FN void unpin() { --npin; }
  KG_FN int clone(int se) {  // StateEventCloner.copyStateEvent:46-58 (shallow)
    pin(se);
    const int c = new_state(false);
    unpin();
    if (c < 0) return -1;
    for (int i = 0; i < nS(); ++i) slot(c, i) = slot(se, i);
    se_ts(c) = se_ts(se);
    return c;
  }
  // copy of the current event (StreamEvent copy with its own `next` link)
  KG_FN int copy_event(int pinned) {
    int n = find_free_nd();
    if (n < 0) {
      pin(pinned);
      gc();
      unpin();
      n = find_free_nd();
      if (n < 0) { cap_fail(CAP_NODES); return -1; }
    }
    nd_used(n >> 6) = (int64_t)((uint64_t)nd_used(n >> 6) | (1ull << (n & 63)));
    nd_seq(n) = seq;
    nd_ts(n) = ts;
    nd_next(n) = -1;
    nd_null(n) = (int32_t)ev_null;
    const int na = q->n_cap[stream];
    for (int j = 0; j < na; ++j) set_nd_val(n, j, ev_val[j]);
    return n;
  }

  // StreamEventPool.borrowEvent()'s empty event (no data, timestamp -1) appended to slot i's chain
  // (StateEvent.addEvent:212-222): an absent logical side whose wait has passed
  KG_FN void add_dummy(int se, int i) {
    pin(se);
    int n = find_free_nd();
    if (n < 0) {
      gc();
      n = find_free_nd();
    }
    unpin();
    if (n < 0) { cap_fail(CAP_NODES); return; }
    nd_used(n >> 6) = (int64_t)((uint64_t)nd_used(n >> 6) | (1ull << (n & 63)));
    nd_seq(n) = -1;
    nd_ts(n) = -1;
    nd_next(n) = -1;
    nd_null(n) = -1;  // every attribute null
    if (slot(se, i) < 0) {
      slot(se, i) = n;
    } else {
      int t = slot(se, i);
      while (nd_next(t) >= 0) t = nd_next(t);
      nd_next(t) = n;
    }
  }

  // ---- lists ----
  KG_FN void nae_push(int i, int se) {
    if (nn(i) >= lay.LC) { cap_fail(CAP_LIST); return; }
    nl(i, nn(i)) = se;
    nn(i) += 1;
  }
  KG_FN void promote(int i) {  // pending.addAll(newAndEvery); newAndEvery.clear()
    if ((flags(i) & FL_ITER) && nn(i) > 0) { fail(GE_REFERENCE); return; }  // Java CME
    const int n = nn(i);
    if (pn(i) + n > lay.LC) { cap_fail(CAP_LIST); return; }
    for (int k = 0; k < n; ++k) pl(i, pn(i) + k) = nl(i, k);
    pn(i) += n;
    nn(i) = 0;
  }

  // ---- pre processors ----
  KG_FN void init_pre(int i) {  // StreamPreStateProcessor.init:157-166
    const GState& s = S(i);
    const bool absent_next = q->type == Q_SEQUENCE && s.next_pre >= 0 && absent_any(s.next_pre);
    if (s.is_start && (!(flags(i) & FL_INIT) || s.next_every >= 0 || absent_next)) {
      const int se = new_state();
      if (se < 0) return;
      add_state(i, se);
      flags(i) |= FL_INIT;
    }
  }
  // addState (StreamPre:203-216 / CountPre:109-132 / LogicalPre:57-76) including the count min-0
  // forwarding chain (CountPost.processMinCountReached:73-85), recursion unrolled: every-targets
  // of the chain are applied deepest first, as the nested calls do
  KG_FN void add_state(int i, int se) {
    int every_t[GMAXS];
    int ne = 0;
    pin(se);
    while (i >= 0) {
      const GState& s = S(i);
      if (s.kind == K_LOGICAL) {
        const int p = s.partner;
        if (absent_l(i) && (flags(i) & FL_INACTIVE)) break;  // AbsentLogicalPre.addState:64-86
        if (s.is_start || q->type == Q_SEQUENCE) {
          if (nn(i) == 0) nae_push(i, se);
          if (nn(p) == 0) nae_push(p, se);
        } else {
          nae_push(i, se);
          nae_push(p, se);
        }
        if (absent_l(i) && !s.is_start && wait_of(i) != -1) {
          notify_at(i, se_ts(se) + wait_of(i));
          if (absent_l(p)) notify_at(p, se_ts(se) + wait_of(p));
        }
        break;
      }
      if (s.kind == K_ABSENT) {  // AbsentStreamPreStateProcessor.addState:78-101
        if (flags(i) & FL_INACTIVE) break;
        if (q->type == Q_SEQUENCE) nn(i) = 0;
        nae_push(i, se);
        if (!s.is_start) {
          lst(i) = se_ts(se) + s.waiting;
          notify_at(i, lst(i));
        }
        break;
      }
      if (q->type == Q_SEQUENCE) {
        if (nn(i) == 0) nae_push(i, se);
      } else {
        nae_push(i, se);
      }
      if (!(s.kind == K_COUNT && s.min == 0 && slot(se, i) < 0)) break;
      // processMinCountReached(i, se)
      if (s.has_selector) {
        flags(i) |= FL_CHANGED;
        flags(i) |= FL_RETURNED;
      }
      if (s.next_every >= 0 && ne < GMAXS) every_t[ne++] = s.next_every;
      i = s.next_pre;
    }
    for (int k = ne - 1; k >= 0; --k) add_every_state(every_t[k], se);
    unpin();
  }
  // addEveryState: StreamPre:218-227 (slot NOT cleared) / LogicalPre:78-92 (both slots cleared)
  KG_FN void add_every_state(int i, int se) {
    const GState& s = S(i);
    const int c = clone(se);
    if (c < 0) return;
    if (s.kind == K_LOGICAL) {
      // AbsentLogicalPreStateProcessor.addEveryState:89-100 keeps the time of its own last event
      if (absent_l(i) && slot(c, i) >= 0) se_ts(c) = nd_ts(slot(c, i));
      slot(c, i) = -1;
      nae_push(i, c);
      slot(c, s.partner) = -1;
      nae_push(s.partner, c);
      return;
    }
    nae_push(i, c);
    if (s.kind == K_ABSENT) {  // AbsentStreamPreStateProcessor.addEveryState:103-115
      lst(i) = se_ts(se) + s.waiting;
      notify_at(i, lst(i));
    }
  }
  // updateState: StreamPre:281-289, CountPre:149-156, LogicalPre:118-130
  KG_FN void update_state(int i) {
    const GState& s = S(i);
    if (s.kind == K_COUNT && (flags(i) & FL_SSRESET)) {
      flags(i) &= ~FL_SSRESET;
      init_pre(i);
    }
    promote(i);
    if (s.kind == K_LOGICAL) promote(s.partner);
  }
  KG_FN bool next_pending_nonempty(int i) {
    const int n = S(i).next_pre;
    if (n < 0) { fail(GE_REFERENCE); return false; }  // NullPointerException in the reference
    return pn(n) > 0;
  }
  // resetState: StreamPre:262-278, LogicalPre:94-116
  KG_FN void reset_state(int i) {
    const GState& s = S(i);
    if (s.kind == K_LOGICAL) {
      const int p = s.partner;
      if (s.ltype == L_OR || pn(i) == pn(p)) {
        pn(i) = 0;
        pn(p) = 0;
        if (s.is_start && nn(i) == 0) {
          if (q->type == Q_SEQUENCE && s.next_every < 0 && next_pending_nonempty(i)) return;
          init_pre(i);
        }
      }
      return;
    }
    pn(i) = 0;
    // AbsentStreamPreStateProcessor.resetState:117-138 re-inits a start state whatever its
    // newAndEvery list holds
    if (s.is_start && (s.kind == K_ABSENT || nn(i) == 0)) {
      if (q->type == Q_SEQUENCE && s.next_every < 0 && next_pending_nonempty(i)) return;
      init_pre(i);
    }
  }
  KG_FN void start_state_reset(int i) {  // CountPreStateProcessor.startStateReset:142-147
    if (S(i).kind != K_COUNT) { fail(GE_REFERENCE); return; }
    flags(i) |= FL_SSRESET;
    if (S(i).callback >= 0) fail(GE_REFERENCE);  // StackOverflowError in the reference
  }
  KG_FN bool is_expired(int i, int se) const {  // StreamPreStateProcessor.isExpired:102-113
    const GState& s = S(i);
    if (s.is_start || within < 0) return false;
    for (int k = 0; k < q->n_start; ++k) {
      const int n = slot(se, q->start_ids[k]);
      if (n >= 0) {
        const int64_t d = (int64_t)((uint64_t)nd_ts(n) - (uint64_t)ts);
        const int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
        if (a > within) return true;
      }
    }
    return false;
  }

  // ---- predicates ----
  KG_FN int chain_at(int head, int64_t idx) const {  // StateEvent.getStreamEvent:138-182
    if (head < 0) return -1;
    if (head == VNODE) return (idx == 0 || idx == -1) ? VNODE : -1;  // one-event chain
    if (idx >= 0) {
      int e = head;
      for (int64_t k = 1; k <= idx; ++k) {
        e = nd_next(e);
        if (e < 0) return -1;
      }
      return e;
    }
    if (idx == -1) {
      int e = head;
      while (nd_next(e) >= 0) e = nd_next(e);
      return e;
    }
    if (idx == -2) {
      if (nd_next(head) < 0) return -1;
      int e = head;
      while (nd_next(nd_next(e)) >= 0) e = nd_next(e);
      return e;
    }
    int64_t len = 0;
    for (int e = head; e >= 0; e = nd_next(e)) ++len;
    int64_t k = len + idx;
    if (k < 0) return -1;
    int e = head;
    for (int64_t j = 0; j < k; ++j) e = nd_next(e);
    return e;
  }
  KG_FN Val run_code(int b, int e, int se) const {
    // shallow programs (a wave-uniform property of the shape) keep the stack in registers
    if (q->max_depth <= RSTACK) return run_code_t<RegStack>(b, e, se);
    return run_code_t<ArrStack>(b, e, se);
  }
  template <class Stack>
  KG_FN Val run_code_t(int b, int e, int se) const {
    return eval_code<Stack>(
        q, ql, b, e,
        [&](const GInsn& in) {  // OP_ATTR: the slot's chain element (CURRENT=-1, LAST=-2, ...)
          const int n = chain_at(slot(se, in.a), in.b);
          Val v{in.res, 1, 0};
          const bool cur = n == VNODE;
          if (n >= 0 && !(((cur ? (int32_t)ev_null : nd_null(n)) >> in.imm) & 1)) {
            v.null = 0;
            const int64_t raw = cur ? ev_val[in.imm] : nd_val(n, (int)in.imm);
            v.bits = in.res == T_INT ? (int64_t)(int32_t)raw : in.res == T_FLOAT ? (int64_t)(uint32_t)raw : raw;
          }
          return v;
        },
        [&](const GInsn& in) { return chain_at(slot(se, in.a), in.b) < 0; });
  }
  KG_FN bool filters_pass(int i, int se) const {  // FilterProcessor.process:55-66
    const GState& s = S(i);
    for (int f = 0; f < s.n_filt; ++f) {
      const Val v = run_code(s.fb[f], s.fe[f], se);
      if (v.null || !v.bits) return false;
    }
    return true;
  }

  // ---- post processors ----
  KG_FN void stream_post(int i, int se) {  // StreamPostStateProcessor.process:53-72
    const GState& s = S(i);
    flags(i) |= FL_CHANGED;
    se_ts(se) = nd_ts(slot(se, i));
    if (s.has_selector) flags(i) |= FL_RETURNED;
    if (s.next_pre >= 0) add_state(s.next_pre, se);
    if (s.next_every >= 0) add_every_state(s.next_every, se);
    if (s.callback >= 0) start_state_reset(s.callback);
  }
  KG_FN void min_count_reached(int i, int se) {  // CountPost.processMinCountReached:73-85
    const GState& s = S(i);
    if (s.has_selector) {
      flags(i) |= FL_CHANGED;
      flags(i) |= FL_RETURNED;
    }
    if (s.next_pre >= 0) add_state(s.next_pre, se);
    if (s.next_every >= 0) add_every_state(s.next_every, se);
  }
  KG_FN void count_post(int i, int se) {  // CountPostStateProcessor.process:45-71
    const GState& s = S(i);
    int e = cnt_tail;
    int64_t n = cnt_len;
    if (e < 0) {
      e = slot(se, i);
      n = 1;
      for (int nx = nd_next(e); nx >= 0; nx = nd_next(e)) { ++n; e = nx; }
    }
    flags(i) |= FL_SUCCESS;
    se_ts(se) = nd_ts(e);
    if (n >= s.min) {
      if (q->type == Q_SEQUENCE) {
        if (s.next_pre >= 0) add_state(s.next_pre, se);
        if (n != s.max) add_state(i, se);
      } else if (n == s.min) {
        min_count_reached(i, se);
      }
      if (n == s.max) flags(i) |= FL_CHANGED;
    }
  }
  // AbsentLogicalPreStateProcessor.partnerCanProceed:342-372 (asked by the partner's AND post)
  KG_FN bool partner_can_proceed(int j, int se) {
    const GState& a = S(j);
    if (q->type == Q_SEQUENCE && a.next_every < 0 && lst(j) > 0) return false;
    if (wait_of(j) == -1) {
      if (a.next_every < 0) return slot(se, j) < 0;
      if (lst(j) > 0) {
        lst(j) = 0;
        init_pre(j);
        return false;
      }
      return true;
    }
    return slot(se, j) >= 0;
  }
  KG_FN void logical_post(int i, int se) {  // LogicalPostStateProcessor.process:59-87
    const GState& s = S(i);
    if (absent_l(i)) {  // AbsentLogicalPostStateProcessor.process:37-49 (lst = lastArrivalTime)
      flags(i) |= FL_CHANGED;
      flags(i) |= FL_RETURNED;
      lst(i) = nd_ts(slot(se, i));
      return;
    }
    if (s.ltype == L_AND) {
      const bool go = absent_l(s.partner) ? partner_can_proceed(s.partner, se) : slot(se, s.partner) >= 0;
      if (go) stream_post(i, se);
      else flags(i) |= FL_CHANGED;
    } else {
      stream_post(i, se);
      if (S(s.partner).has_selector && s.this_last == s.partner) flags(s.partner) |= FL_RETURNED;
    }
  }
  // AbsentStreamPostStateProcessor.process:31-52: the absent event arrived -- the partial is dropped
  // and the waiting restarts from this event (AbsentStreamPre.updateLastArrivalTime:69-75)
  KG_FN void absent_post(int i, int se) {
    const GState& s = S(i);
    flags(i) |= FL_CHANGED;
    const int64_t t = nd_ts(slot(se, i));
    se_ts(se) = t;
    flags(i) |= FL_RETURNED;
    if (s.is_start && s.next_every == i) add_every_state(i, se);
    lst(i) = t + s.waiting;
    notify_at(i, lst(i));
  }
  KG_FN void process(int i, int se, bool deferred) {  // deferred: slot i holds VNODE
    flags(i) &= ~FL_CHANGED;
    if (!filters_pass(i, se)) return;
    if (deferred) {  // the filters passed: copy the current event now
      slot(se, i) = -1;
      const int ev = copy_event(se);
      if (ev < 0) return;  // capacity (err is set; the push fails)
      slot(se, i) = ev;
    }
    switch (S(i).kind) {
      case K_STREAM: stream_post(i, se); break;
      case K_ABSENT: absent_post(i, se); break;
      case K_COUNT: count_post(i, se); break;
      default: logical_post(i, se); break;
    }
  }
  KG_FN bool take_returned(int i) {
    const int tl = S(i).this_last;
    if (tl < 0) return false;
    if (flags(tl) & FL_RETURNED) {
      flags(tl) &= ~FL_RETURNED;
      return true;
    }
    return false;
  }
  KG_FN void push_ret(int se) {
    if (n_ret >= lay.LC) { cap_fail(CAP_LIST); return; }
    ret_at(n_ret++) = se;
  }

  // AbsentLogicalPreStateProcessor.processAndReturn:246-300: an arriving event of the absent side
  // marks the partial (its lastArrivalTime moves); the chunk returned is always empty
  KG_FN void absent_logical_par(int i) {
    const GState& s = S(i);
    if (flags(i) & FL_INACTIVE) return;
    flags(i) |= FL_ITER;
    int w = 0;
    const int n0 = pn(i);
    int k = 0;
    for (; k < n0 && err == GE_OK; ++k) {
      const int se = pl(i, k);
      pin(se);
      bool keep = true;
      if (is_expired(i, se)) {
        keep = false;
        if (s.within_every >= 0) {
          add_every_state(s.within_every, se);
          update_state(s.within_every);
        }
      } else if (s.ltype == L_OR && slot(se, s.partner) >= 0) {
        keep = false;
      } else {
        const int cur = slot(se, i);
        slot(se, i) = VNODE;  // copied into the pool by process() once the filters pass
        process(i, se, true);
        if (wait_of(i) != -1 || (q->type == Q_SEQUENCE && s.ltype == L_AND && s.next_every >= 0)) slot(se, i) = cur;
        bool removed = false;
        if (take_returned(i)) {  // no longer an absent candidate
          keep = false;
          removed = true;
          if (q->type == Q_SEQUENCE) remove_first(s.partner, se);
        }
        if (!(flags(i) & FL_CHANGED)) {
          slot(se, i) = cur;
          if (q->type == Q_SEQUENCE) {
            if (removed) fail(GE_REFERENCE);  // IllegalStateException (second iterator.remove)
            keep = false;
          }
        }
      }
      unpin();
      if (keep) pl(i, w++) = se;
    }
    for (; k < n0; ++k) pl(i, w++) = pl(i, k);  // not visited (error): kept
    pn(i) = w;
    flags(i) &= ~FL_ITER;
  }
  KG_FN void remove_first(int j, int se) {  // pendingStateEventList.remove(Object)
    const int n = pn(j);
    for (int k = 0; k < n; ++k)
      if (pl(j, k) == se) {
        for (int m = k + 1; m < n; ++m) pl(j, m - 1) = pl(j, m);
        pn(j) = n - 1;
        return;
      }
  }

  // processAndReturn: StreamPre:292-337, CountPre:53-93, LogicalPre:133-178. Emitted partials
  // are collected in `ret` (GC roots) and handed to the emitter after the loop, as the reference
  // returns its ComplexEventChunk.
  KG_FN void process_and_return(int i) {
    const GState& s = S(i);
    if (s.kind == K_ABSENT && (flags(i) & FL_INACTIVE)) return;  // AbsentStreamPre.processAndReturn:231-244
    if (absent_l(i)) { absent_logical_par(i); return; }
    flags(i) |= FL_ITER;
    int w = 0;
    const int nS_ = nS();
    const int n0 = pn(i);
    int k = 0;
    for (; k < n0 && err == GE_OK; ++k) {
      const int se = pl(i, k);
      pin(se);
      bool keep = true;
      if (s.kind == K_COUNT) {
        if ((nS_ > i + 1 && slot(se, i + 1) >= 0) || (nS_ > i + 2 && slot(se, i + 2) >= 0)) {
          keep = false;
        } else {
          const int ev = copy_event(se);
          if (ev < 0) { unpin(); break; }
          int prev = -1;  // the node before ev
          int64_t len = 1;
          if (slot(se, i) < 0) slot(se, i) = ev;  // StateEvent.addEvent:212-222
          else {
            int t = slot(se, i);
            len = 2;
            for (int nx = nd_next(t); nx >= 0; nx = nd_next(t)) { t = nx; ++len; }
            nd_next(t) = ev;
            prev = t;
          }
          flags(i) &= ~FL_SUCCESS;
          cnt_tail = ev;
          cnt_len = len;
          process(i, se, false);
          cnt_tail = -1;
          if (take_returned(i)) push_ret(se);
          bool removed = false;
          if (flags(i) & FL_CHANGED) { keep = false; removed = true; }
          if (!(flags(i) & FL_SUCCESS)) {
            // StateEvent.removeLastEvent:224-236. The filters failed, so nothing ran between the
            // append and here and ev is still the chain's last node: unlink it from prev
            if (prev >= 0) nd_next(prev) = -1;
            else slot(se, i) = -1;
            if (q->type == Q_SEQUENCE) {
              if (removed) fail(GE_REFERENCE);  // IllegalStateException (second iterator.remove)
              keep = false;
            }
          }
        }
      } else if (is_expired(i, se)) {
        keep = false;
        if (s.within_every >= 0) {
          add_every_state(s.within_every, se);
          update_state(s.within_every);
        }
      } else if (s.kind == K_LOGICAL && s.ltype == L_OR && slot(se, s.partner) >= 0) {
        keep = false;
      } else {
        slot(se, i) = VNODE;  // copied into the pool by process() once the filters pass
        process(i, se, true);
        // an absent processor always returns an empty chunk
        if (take_returned(i) && s.kind != K_ABSENT) push_ret(se);
        if (flags(i) & FL_CHANGED) {
          keep = false;
        } else {
          slot(se, i) = -1;
          if (q->type == Q_SEQUENCE) {
            // removeOnNoStateChange: true for StreamPre, false for AbsentStreamPre (:246-248)
            if (s.kind != K_ABSENT) keep = false;
            if ((s.kind == K_STREAM || s.kind == K_ABSENT) && s.callback >= 0) start_state_reset(s.callback);
          }
        }
      }
      unpin();
      if (keep) pl(i, w++) = se;
    }
    for (; k < n0; ++k) pl(i, w++) = pl(i, k);  // not visited (error): kept
    pn(i) = w;
    flags(i) &= ~FL_ITER;
  }

  // one event of this instance's streams (Runtime.receive: SingleProcessStreamReceiver.java:57-80,
  // MultiProcessStreamReceiver.receive:268-279 + StateMultiProcessStreamReceiver:53-74; sequences
  // reset and update the whole runtime first, StateStreamRuntime.java:89-92)
  template <class Emit>
  KG_FN void receive(Emit& em) {
    const int sidx = stream;
    const int np = q->recv_n[sidx];
    if (np == 0) return;
    if (q->type == Q_SEQUENCE) {
      for (int k = 0; k < q->n_reset; ++k) reset_state(q->reset_order[k]);
      for (int k = 0; k < q->n_update; ++k) update_state(q->update_order[k]);
    } else {
      for (int k = 0; k < np; ++k) update_state(q->recv_procs[sidx][k]);
    }
    for (int k = np - 1; k >= 0 && err == GE_OK; --k) {  // reverse registration order
      n_ret = 0;
      process_and_return(q->recv_procs[sidx][k]);
      for (int r = 0; r < n_ret; ++r) em(*this, ret_at(r));
      n_ret = 0;
    }
  }
  KG_FN void init_instance() {  // QueryRuntime.init -> node_init(0)
    for (int k = 0; k < q->n_init; ++k) init_pre(q->init_order[k]);
  }
  // SiddhiAppRuntime.start -> AbsentStreamPreStateProcessor.start:276-286: start states with a
  // 'for' time schedule their first check at the runtime's start time
  KG_FN void start_instance(int64_t start_ts) {
    if (lay.TQ == 0) return;
    for (int i = 0; i < lay.S; ++i) {
      const GState& s = S(i);
      if (s.kind == K_ABSENT && s.is_start && s.waiting != -1 && !(flags(i) & FL_INACTIVE)) {
        lst(i) = start_ts + s.waiting;
        notify_at(i, lst(i));
      }
      // AbsentLogicalPreStateProcessor.start:320-330
      if (absent_l(i) && s.is_start && wait_of(i) != -1 && !(flags(i) & FL_INACTIVE)) notify_at(i, start_ts + wait_of(i));
    }
  }

  // AbsentStreamPreStateProcessor.sendEvent:212-228
  template <class Emit>
  KG_FN void absent_send(int i, int se, Emit& em) {
    const GState& s = S(i);
    if (s.has_selector) em(*this, se);  // thisStatePostProcessor.nextProcessor: the selector
    if (s.next_pre >= 0) add_state(s.next_pre, se);
    if (s.next_every >= 0) add_every_state(s.next_every, se);
    else if (s.is_start) flags(i) |= FL_INACTIVE;
    if (s.callback >= 0) start_state_reset(s.callback);
  }
  // AbsentStreamPreStateProcessor.process:140-210: a timer event of state i's scheduler at time t
  // (`actual`: the timestamp generator's time -- t itself, or in playback the event time that let
  // the timer fire)
  template <class Emit>
  KG_FN void absent_timer(int i, int64_t t, int64_t actual, Emit& em) {
    const GState& s = S(i);
    if (flags(i) & FL_INACTIVE) return;
    bool initialize = s.is_start && nn(i) == 0 && pn(i) == 0;
    if (initialize && q->type == Q_SEQUENCE && s.next_every < 0 && lst(i) > 0) initialize = false;
    if (initialize) {
      const int se = new_state();
      if (se < 0) return;
      add_state(i, se);
    } else if (q->type == Q_SEQUENCE && nn(i) > 0) {
      reset_state(i);
    }
    update_state(i);
    n_ret = 0;
    int w = 0;
    const int n0 = pn(i);
    int k = 0;
    for (; k < n0 && err == GE_OK; ++k) {
      const int se = pl(i, k);
      if (is_expired(i, se)) {  // (ts == t here)
        if (s.within_every >= 0 && s.next_every != i) {
          if (s.next_every < 0) { fail(GE_REFERENCE); continue; }  // NullPointerException
          add_every_state(s.next_every, se);
        }
        continue;
      }
      const int64_t st = se_ts(se);
      if ((st == -1 && t >= lst(i)) || (st != -1 && t >= st + s.waiting)) {
        se_ts(se) = t;
        push_ret(se);
        continue;
      }
      pl(i, w++) = se;
    }
    for (; k < n0; ++k) pl(i, w++) = pl(i, k);  // not visited (error): kept
    pn(i) = w;
    if (s.within_every >= 0) update_state(s.within_every);
    const bool not_processed = n_ret == 0;
    for (int r = 0; r < n_ret && err == GE_OK; ++r) absent_send(i, ret_at(r), em);
    n_ret = 0;
    if (actual > s.waiting + t) lst(i) = actual + s.waiting;
    if (not_processed && lst(i) < t) {
      lst(i) = t + s.waiting;
      notify_at(i, lst(i));
    }
  }
  // AbsentLogicalPreStateProcessor.sendEvent:225-244
  template <class Emit>
  KG_FN void absent_logical_send(int i, int se, Emit& em) {
    const GState& s = S(i);
    if (s.has_selector) em(*this, se);
    if (s.next_pre >= 0) add_state(s.next_pre, se);
    if (s.next_every >= 0) {
      add_every_state(s.next_every, se);
    } else if (s.is_start) {
      flags(i) |= FL_INACTIVE;
      if (s.ltype == L_OR && absent_l(s.partner)) flags(s.partner) |= FL_INACTIVE;
    }
    if (s.callback >= 0) start_state_reset(s.callback);
  }
  // AbsentLogicalPreStateProcessor.process:107-181: a timer of logical side i at time t
  template <class Emit>
  KG_FN void absent_logical_timer(int i, int64_t t, int64_t actual, Emit& em) {
    const GState& s = S(i);
    if (flags(i) & FL_INACTIVE) return;
    const int64_t w = wait_of(i);
    bool not_processed = true;
    if (t >= lst(i) + w) {
      if (s.is_start && q->type == Q_SEQUENCE && nn(i) == 0 && pn(i) == 0) {
        const int se = new_state();
        if (se < 0) return;
        add_state(i, se);
      } else if (q->type == Q_SEQUENCE && nn(i) > 0) {
        reset_state(i);
      }
      update_state(i);
      n_ret = 0;
      int wr = 0;
      const int n0 = pn(i);
      int k = 0;
      for (; k < n0 && err == GE_OK; ++k) {
        const int se = pl(i, k);
        if (is_expired(i, se)) {  // (ts == t here)
          if (s.within_every >= 0) {
            add_every_state(s.within_every, se);
            update_state(s.within_every);
          }
          continue;
        }
        const int own = slot(se, i);
        const bool passed = own < 0 ? t >= se_ts(se) + w : t >= nd_ts(own) + w;  // waitingTimePassed
        if (!passed) {
          pl(i, wr++) = se;
          continue;
        }
        const bool partner = slot(se, s.partner) >= 0;
        if (s.ltype == L_OR && !partner) {
          add_dummy(se, i);
          push_ret(se);
        } else if (s.ltype == L_AND && partner) {
          push_ret(se);
        } else if (s.ltype == L_AND && !partner) {
          pin(se);
          add_dummy(se, i);  // the partner may still proceed
          unpin();
        }
      }
      for (; k < n0; ++k) pl(i, wr++) = pl(i, k);
      pn(i) = wr;
      not_processed = n_ret == 0;
      for (int r = 0; r < n_ret && err == GE_OK; ++r) absent_logical_send(i, ret_at(r), em);
      n_ret = 0;
      lst(i) = 0;
    }
    if (s.next_every >= 0 || (not_processed && s.is_start)) notify_at(i, (lst(i) == 0 ? actual : lst(i)) + w);
  }
  // the earliest pending notification time of the instance's schedulers (INT64_MAX: none)
  KG_FN int64_t next_due() const {
    int64_t d = 0x7fffffffffffffffLL;
    if (lay.TQ == 0) return d;
    for (int i = 0; i < lay.S; ++i) {
      if (!absent_any(i) || tq_len(i) == 0) continue;
      const int64_t h = tq(i, tq_head(i));
      d = h < d ? h : d;
    }
    return d;
  }
  // Scheduler.sendTimerEvents:186-214 of every absent state of the instance up to time `upto`: the
  // earliest queue head fires first (ties: lower state id). `playback`: the generator's time is
  // `upto` while the timers fire; else each timer's own time.
  template <class Emit>
  KG_FN void fire_timers(int64_t upto, bool playback, Emit& em) {
    if (lay.TQ == 0) return;
    const int64_t ev_ts = ts;
    // the sort key of this call's timer matches: the running max of the fired times. The oracle
    // fires across instances by smallest queue head; a FIFO can hold a time behind a later one, and
    // that one fires right after it, so (running max, query, fire order) is the global fire order
    int64_t key = -0x7fffffffffffffffLL - 1;
    for (;;) {
      int bi = -1;
      int64_t bt = 0;
      for (int i = 0; i < lay.S; ++i) {
        if (!absent_any(i) || tq_len(i) == 0) continue;
        const int64_t h = tq(i, tq_head(i));
        if (h > upto) continue;
        if (bi < 0 || h < bt) {
          bi = i;
          bt = h;
        }
      }
      if (bi < 0 || err != GE_OK) break;
      tq_head(bi) = (tq_head(bi) + 1) % lay.TQ;
      tq_len(bi) -= 1;
      in_timer = true;
      key = bt > key ? bt : key;
      timer_ts = key;
      ts = bt;
      if (absent_l(bi)) absent_logical_timer(bi, bt, playback ? upto : bt, em);
      else absent_timer(bi, bt, playback ? upto : bt, em);
      in_timer = false;
    }
    ts = ev_ts;
  }
};

// ------------------------------------------------------------------------------------------
// host-side layout of one query's arenas
// ------------------------------------------------------------------------------------------
inline void make_layout(GLayout& L, int S, int R, int N, int LC, int NA, bool v32 = false, int TQ = 0) {
  L.S = S; L.R = R; L.N = N; L.LC = LC; L.NA = NA; L.NU = (N + 63) / 64;
  L.SU = (R + 63) / 64;
  L.big = (L.SU > 1 || L.NU > GMAXNU) ? 1 : 0;
  L.pad = 0;
  L.v32 = v32 ? 1 : 0;
  int o = 0;
  L.o_flags = o; o += S;
  L.o_pn = o; o += S;
  L.o_nn = o; o += S;
  L.o_plist = o; o += S * LC;
  L.o_nlist = o; o += S * LC;
  L.o_seslot = o; o += R * S;
  L.o_ndnext = o; o += N;
  L.o_ndnull = o; o += N;
  L.o_init = o; o += 1;
  if (v32) { L.o_ndval = o; o += N * NA; }
  L.TQ = TQ;
  L.o_tqh = o; o += TQ > 0 ? 2 * S : 0;
  L.o_ret = o; o += LC;
  L.pad2 = 0;
  L.n32 = o;
  o = 0;
  L.o_seused = o; o += L.SU;
  L.o_ndused = o; o += L.NU;
  L.o_mark = o; o += L.big ? L.SU + L.NU : 0;
  L.o_sets = o; o += R;
  L.o_ndseq = o; o += N;
  L.o_ndts = o; o += N;
  if (!v32) { L.o_ndval = o; o += N * NA; }
  L.o_tq = o; o += S * TQ;
  L.o_lst = o; o += TQ > 0 ? S : 0;
  L.n64 = o;
}

// Events of look-back that rebuild this query's state exactly at any point of a batch, or -1.
// A SEQUENCE of stream states whose start re-arms itself (`every e1, e2, ...`) resets every pending
// list before each event (R14, StateStreamRuntime.java:89-92) and drops a partial at its first
// non-matching event (R6e), so a partial alive before event k was opened at most S-1 events
// earlier, and the start state always holds one partial whose slots are overwritten before they
// are read (a fresh seed is equivalent). The state before event k is therefore a function of
// events k-S+1 .. k-1 alone: an event chunk can start from a fresh instance and replay S-1 events.
inline int seq_lookback(const GQuery& g) {
  if (g.type != Q_SEQUENCE) return -1;
  int st0 = -1, n0 = 0;  // (start_ids lists the start states only for `within` checks)
  for (int i = 0; i < g.n_states; ++i)
    if (g.st[i].is_start) st0 = i, ++n0;
  if (n0 != 1 || g.st[st0].next_every != st0) return -1;
  for (int i = 0; i < g.n_states; ++i) {  // (a start state never expires: its within-every is inert)
    const GState& s = g.st[i];
    if (s.kind != K_STREAM || (s.within_every >= 0 && !s.is_start) || s.callback >= 0) return -1;
  }
  return g.n_states - 1;
}

// K_seq: a look-back sequence whose states all read one stream, chained 0 -> 1 -> ... -> S-1.
// Then a partial alive at state j before event k was opened at event k-j and its slots are events
// k-j .. k-1, so a match is a property of a window of S consecutive events alone: starting at s,
// every state i passes its filters over events s .. s+i, and no step i >= 1 is expired
// (|ts[s] - ts[s+i]| > within). Returns S, or -1.
inline int code_depth(const GQuery& g, int b, int e) {  // max evaluation-stack entries of a range
  int sp = 0, mx = 0;
  for (int pc = b; pc < e; ++pc) {
    const int op = g.code[pc].op;
    if (op == OP_CONST || op == OP_ATTR || op == OP_STREAM_IS_NULL) ++sp;
    else if (op == OP_AND || op == OP_OR || op == OP_CMP || op == OP_ARITH) --sp;
    else if (op != OP_IS_NULL && op != OP_NOT) ++sp;
    mx = sp > mx ? sp : mx;
  }
  return mx;
}

inline int seq_window(const GQuery& g) {
  if (seq_lookback(g) < 0) return -1;
  for (int i = 0; i < g.n_states; ++i)
    for (int f = 0; f < g.st[i].n_filt; ++f)
      if (code_depth(g, g.st[i].fb[f], g.st[i].fe[f]) > RSTACK) return -1;
  const int st = g.st[0].stream;
  if (!g.st[0].is_start) return -1;
  for (int i = 0; i < g.n_states; ++i)
    if (g.st[i].stream != st || g.st[i].next_pre != (i + 1 < g.n_states ? i + 1 : -1)) return -1;
  for (int k = 0; k < GMAXSTREAM; ++k)
    if (k != st && g.recv_n[k] != 0) return -1;
  return g.n_states;
}

// One window of a K_seq query: does the sequence started at window event 0 match events 0 .. S-1?
// Win provides ts(p) and, for event p and captured attribute word j, raw(p, j) / null(p, j). Slots
// hold one event each, so eK / eK[0] / eK[last] name it and every other index is null
// (StateEvent.getStreamEvent:138-182 on a one-event chain); state i's filter sees slots 0 .. i.
// the lane's constant of a CONST leaf: its query's bytecode immediate, or (Win::lane_const) a copy
// the device kernel staged in LDS once per work item
template <class Win>
KG_FN int64_t leaf_const(const GLeaf& f, const GQuery* ql, const Win& w) {
  if constexpr (Win::kStagedConsts) return w.lane_const(f.cslot);
  else return ql->code[f.pc].imm;
}

template <class Win>
KG_FN Val atom_leaf(const GLeaf& f, const GQuery* ql, const Win& w) {
  Val v{f.type, 1, 0};
  if (f.kind == LF_CONST) {
    const int64_t imm = leaf_const(f, ql, w);
    v.null = 0;
    v.bits = f.type == T_FLOAT ? (int64_t)(uint32_t)imm : f.type == T_INT ? (int64_t)(int32_t)imm : imm;
  } else if ((f.kind == LF_ATTR || f.kind == LF_ATTR0) && !w.null(f.slot, f.cap, f.kind == LF_ATTR0)) {
    const int64_t raw = w.raw(f.slot, f.cap, f.kind == LF_ATTR0);
    v.null = 0;
    v.bits = f.type == T_INT ? (int64_t)(int32_t)raw : f.type == T_FLOAT ? (int64_t)(uint32_t)raw : raw;
  }
  return v;
}
template <class Win>
KG_FN Val atom_opnd(const GOpnd& o, const GQuery* ql, const Win& w) {
  Val a = atom_leaf(o.a, ql, w);
  if (o.arith < 0) return a;
  return arith(o.arith, o.res, a, atom_leaf(o.b, ql, w));
}
// the atoms of state i over window w (FilterProcessor + the typed compare / arithmetic executors)
template <class Win>
KG_FN bool atoms_pass(const GQuery* q, const GQuery* ql, int i, const Win& w) {
  for (int t = q->atom_begin[i]; t < q->atom_begin[i + 1]; ++t) {
    const GAtom& A = q->atoms[t];
    Val l = atom_opnd(A.l, ql, w), r = atom_opnd(A.r, ql, w);
    l.type = A.lt;
    r.type = A.rt;
    if (l.null || r.null || !typed_compare(A.op, l, r)) return false;
  }
  return true;
}

// (n_st >= 0: only states 0 .. n_st-1, i.e. a partial waiting at state n_st -- live-partial counts)
template <class Win>
KG_FN bool seq_match(const GQuery* q, const GQuery* ql, int64_t within, const Win& w, int n_st = -1) {
  const int S = n_st < 0 ? q->n_states : n_st;
  for (int i = 0; i < S; ++i) {
    if (i >= 1 && within >= 0) {  // StreamPreStateProcessor.isExpired:102-113 before the filter
      const int64_t d = (int64_t)((uint64_t)w.ts(0) - (uint64_t)w.ts(i));
      const int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
      if (a > within) return false;
    }
    if (q->n_atoms != 0) {  // the shape's filters are atoms (wave-uniform choice)
      if (!atoms_pass(q, ql, i, w)) return false;
      continue;
    }
    const GState& st = q->st[i];
    for (int f = 0; f < st.n_filt; ++f) {
      const Val v = eval_code<RegStack>(
          q, ql, st.fb[f], st.fe[f],
          [&](const GInsn& in) {
            Val x{in.res, 1, 0};
            if (in.a <= i && (in.b == 0 || in.b == -1) && !w.null(in.a, (int)in.imm)) {
              x.null = 0;
              const int64_t raw = w.raw(in.a, (int)in.imm);
              x.bits = in.res == T_INT ? (int64_t)(int32_t)raw : in.res == T_FLOAT ? (int64_t)(uint32_t)raw : raw;
            }
            return x;
          },
          [&](const GInsn& in) { return !(in.a <= i && (in.b == 0 || in.b == -1)); });
      if (v.null || !v.bits) return false;
    }
  }
  return true;
}

// Lower every filter of g to compare atoms (K_seq windows, seq_match): a filter must be an AND tree
// of compares whose operands are leaves or one arithmetic op over two leaves. A slot reference
// names state a's one event when a <= the filter's state and the chain index is 0 / CURRENT (a
// window slot holds one event, StateEvent.getStreamEvent:138-182), and reads null otherwise.
// Leaves g.n_atoms = 0 when some filter has another form (or / not / is null / deeper arithmetic).
inline void lower_atoms(GQuery& g) {
  g.n_atoms = 0;
  g.n_const = 0;
  int na = 0;
  for (int i = 0; i < g.n_states; ++i) {
    g.atom_begin[i] = na;
    const GState& st = g.st[i];
    for (int f = 0; f < st.n_filt; ++f) {
      // postfix -> tree: node = instruction index, children by stack simulation
      int stk[GSTACK], sp = 0, left[GMAXCODE], right[GMAXCODE];
      for (int pc = st.fb[f]; pc < st.fe[f]; ++pc) {
        const GInsn& in = g.code[pc];
        left[pc] = right[pc] = -1;
        if (in.op == OP_CONST || in.op == OP_ATTR) {
          if (sp >= GSTACK) return;
          stk[sp++] = pc;
        } else if (in.op == OP_CMP || in.op == OP_AND || in.op == OP_ARITH) {
          if (sp < 2) return;
          right[pc] = stk[--sp];
          left[pc] = stk[--sp];
          stk[sp++] = pc;
        } else {
          return;  // or / not / is null / stream is null: interpreter
        }
      }
      if (sp != 1) return;
      int todo[GMAXCODE], nt = 0;
      todo[nt++] = stk[0];
      while (nt) {
        const int x = todo[--nt];
        const GInsn& in = g.code[x];
        if (in.op == OP_AND) {
          todo[nt++] = right[x];  // left conjunct first (short-circuit order does not matter: pure)
          todo[nt++] = left[x];
          continue;
        }
        if (in.op != OP_CMP || na >= GMAXATOM) return;
        GAtom& A = g.atoms[na++];
        A = GAtom{};
        A.state = (int8_t)i;
        A.op = (int8_t)in.imm;
        A.lt = in.lt;
        A.rt = in.rt;
        auto leaf = [&](int pc, GLeaf& L) -> bool {
          const GInsn& li = g.code[pc];
          L = GLeaf{};
          L.type = li.res;
          if (li.op == OP_CONST) {
            if (g.n_const >= GMAXCONST) return false;
            L.kind = LF_CONST;
            L.pc = (int16_t)pc;
            L.cslot = (int16_t)g.n_const;
            g.const_pc[g.n_const++] = pc;
            return true;
          }
          if (li.op != OP_ATTR) return false;
          const bool here = li.a <= i && (li.b == 0 || li.b == -1);
          L.kind = here ? (li.b == 0 ? LF_ATTR0 : LF_ATTR) : LF_NULL;
          L.slot = (int8_t)li.a;
          L.cap = (int8_t)li.imm;
          return true;
        };
        auto opnd = [&](int pc, GOpnd& O) -> bool {
          O = GOpnd{};
          O.arith = -1;
          const GInsn& oi = g.code[pc];
          if (oi.op != OP_ARITH) return leaf(pc, O.a);
          O.arith = (int8_t)oi.imm;
          O.res = oi.res;
          if (!leaf(left[pc], O.a) || !leaf(right[pc], O.b)) return false;
          O.a.type = oi.lt;  // eval_code types arithmetic operands from the instruction
          O.b.type = oi.rt;
          return true;
        };
        if (!opnd(left[x], A.l) || !opnd(right[x], A.r)) return;
      }
    }
  }
  g.atom_begin[g.n_states] = na;
  for (int i = g.n_states + 1; i <= GMAXS; ++i) g.atom_begin[i] = na;
  g.n_atoms = na > 0 ? na : -1;  // -1: atoms lowered, none needed (filterless states)
}
inline void lower_atoms_or_none(GQuery& g) {
  lower_atoms(g);
  if (g.n_atoms == 0) g.n_const = 0;
}

// Shape of a query: the lowered program with what may differ between lanes of one wave cleared
// (qid, rank, the `within` value -- its presence stays -- and bytecode constants). Queries with
// equal shapes share one wave-uniform template on the device.
inline GQuery shape_of(const GQuery& g) {
  GQuery s = g;
  s.qid = 0;
  s.rank = 0;
  s.within = g.within < 0 ? -1 : 0;
  for (int pc = 0; pc < s.n_code; ++pc)
    if (s.code[pc].op == OP_CONST) s.code[pc].imm = 0;
  return s;
}

}  // namespace kg
}  // namespace sdh
