// nfa_types.h -- device-visible program tables of the MI355X NFA engine (host + device).
//
// A query of the "chain" family (every? s0 -> s1 -> ... -> s{n-1} [within T], stream states
// only) is lowered to a ChainQuery: per state its stream and a conjunction of compare atoms
// (the predicate bytecode), plus the captured attribute values later filters read
// (e.g. e1.price for `price > e1.price`). Device kernels read these tables through the scalar
// cache (all fields are wave-uniform).
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#endif

namespace sdh {

constexpr int MAXS = 4;      // states per chain query
constexpr int MAXCAP = 4;    // captured operand keys per partial match
constexpr int MAXATOM = 12;  // compare atoms per query (all states)
constexpr int MAXCOL = 8;    // pre-keyed operand columns of the current event
constexpr int MAXXA = 4;     // atoms reading captured values (evaluated per partial)
constexpr int MAXATTR = 16;  // attributes per stream
constexpr int WAVE = 64;

enum AttrType { T_INT = 0, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_STRING };
// compare domain = the precision Java evaluates the typed compare in
enum Domain { D_I32 = 0, D_I64, D_F32, D_F64, D_RAW };
// operand kinds
enum OpKind { OPK_CUR = 0, OPK_CAP, OPK_CONST, OPK_NULL };
enum CmpOp { CMP_EQ = 0, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE };

// Key conversions: an attribute value is converted ONCE (per event, when its tile is staged, or
// per capture) into the key of its compare domain, so that every compare is a plain f64 or i64
// compare. F32-domain values are rounded to binary32 first and then widened exactly, so comparing
// the f64 keys gives Java's float compare bit-for-bit (NaN included).
enum Conv {
  CV_I64_INT = 0,   // (long) int
  CV_I64_LONG,      // long
  CV_F32_INT,       // (double)(float) int
  CV_F32_LONG,      // (double)(float) long
  CV_F32_FLOAT,     // (double) float
  CV_F64_INT,       // (double) int
  CV_F64_LONG,      // (double) long
  CV_F64_FLOAT,     // (double) float
  CV_F64_DOUBLE,    // double
  CV_RAW,           // bool / string id
};

// compare result = ((lt & b0) | (gt & b1) | (eq & b2)) ^ b3
enum CmpMask { CM_LT = 1, CM_GT = 2, CM_EQ = 4, CM_NOT = 8 };

struct Atom {
  int32_t mask;         // CmpMask bits
  int32_t f64;          // 1: compare keys as double, 0: as int64
  int32_t lk, li;       // lhs kind, column (CUR) / capture (CAP) index
  int32_t rk, ri;
  int64_t lc, rc;       // constant keys (CONST)
};

struct ChainQuery {
  int32_t qid;          // index of the query in the program
  int32_t n_states;
  int32_t every;        // 1: `every` on the start state
  int32_t n_cap;
  int64_t within;       // ms, -1 = no within
  int32_t chunkable;    // planner proof that warm-up chunking is exact
  int32_t n_col;        // pre-keyed operand columns
  int32_t col_attr[MAXCOL], col_conv[MAXCOL], col_stream[MAXCOL];
  int32_t state_stream[MAXS];
  // atoms of state s are [atom_begin[s], atom_begin[s+1]); those that read captured values are
  // listed as "x-atoms" xa_first[s] .. xa_first[s]+xa_count[s]-1 (xa_atom[j] = atom index) and
  // evaluated per partial; all others read only the current event and constants and are
  // evaluated for a whole 64-event tile at once (one lane per event).
  int32_t atom_begin[MAXS + 1];
  int32_t xa_first[MAXS], xa_count[MAXS];
  int32_t n_xa;
  int32_t xa_atom[MAXXA];      // atom index of x-atom j
  int32_t xa_col[MAXXA];       // column of its current-event operand (-1: none)
  int32_t cap_slot[MAXCAP], cap_col[MAXCAP];
  Atom atoms[MAXATOM];
};

// one wave of the NFA-step launch = one (query instance, event chunk)
struct WorkItem {
  int32_t q;            // index into the ChainQuery table
  int32_t chunk, n_chunks;
  int32_t inb;          // which of the two state buffers holds the instance's current state
  int64_t c0, c1;       // events of the batch whose emissions this item owns
  int64_t seg_off;      // first match record of this item's output segment
  int64_t seg_cap;      // capacity of the segment (records)
};

// persisted partial-match table of one query instance: NF fields x PCAP lanes (SoA, int64)
enum Field { F_STATE = 0, F_TS0, F_SEQ0, F_SEQ1, F_SEQ2, F_CAP0, F_CAP1, F_CAP2, F_CAP3, F_CAPNULL, NF };
static_assert(F_SEQ0 + MAXS - 1 == F_CAP0, "seq fields");
static_assert(F_CAP0 + MAXCAP == F_CAPNULL, "cap fields");

struct InstHeader {
  int32_t seed_alive;   // start state still holds its seed (non-every patterns consume it)
  int32_t n_live;       // live partials
  int32_t overflow;     // partial table overflowed
  int32_t unordered;    // batch timestamps not monotone (chunked items must be re-run)
};

struct StreamBatch {
  const int64_t* ts;
  const void* col[MAXATTR];
  const uint8_t* nul[MAXATTR];
  int32_t width[MAXATTR];   // bytes per element (4 or 8; bool 1)
  int32_t n_attr;
  int32_t stream;
  int64_t n;
  int64_t seq_base;         // global sequence number of event 0
  int64_t prev_ts;          // last timestamp of the previous batch of this stream (INT64_MIN: none)
};

struct ChainLaunch {
  const ChainQuery* queries;
  const WorkItem* work;
  int32_t n_work;
  int32_t pcap;             // partial capacity per instance (64 * K)
  StreamBatch b;
  InstHeader* hdr[2];       // double-buffered instance headers  [q]
  int64_t* part[2];         // double-buffered partial tables     [q][NF][pcap]
  int64_t* match;           // records of rec_words int64
  int32_t rec_words;
  int32_t pad;
  int64_t* seg_count;       // per work item: matches written
  int32_t* err;             // [0] overflow, [1] unordered, [2] segment overflow
};

// ------------------------------------------------------------------------------------------
// K_ratchet: the 2-state threshold-ratchet family
//     every e1=S[f0] -> e2=S[cur.a OP e1.a] within T        OP in {<, <=, >, >=}
// One lane per pattern; 64 same-shape patterns per wave group. Per lane the pending partials of
// state 1 form a deque ordered by insertion whose keys (e1.a in the x-atom's compare domain) are
// monotone, so each event costs O(1) amortised: expire from the bottom, match from the top, push.
// ------------------------------------------------------------------------------------------
constexpr int RMAXF0 = 4;     // f0 atoms (event-only, per-lane constant operand)
constexpr int RSMAX = 512;    // initial persisted deque capacity per lane (>= LDS ring + spill ring;
                              // the engine doubles it with the spill ring: RatchetLaunch::rsmax)

enum KeyKind { KK_F32 = 0, KK_I32, KK_F64, KK_I64 };

struct RatchetAtom {
  int32_t attr, conv;    // current-event operand: attribute and key conversion
  int32_t cur_left;      // 1: `cur OP const`, 0: `const OP cur`
  int32_t mask;          // CmpMask
  int32_t f64;           // compare keys as double
  int32_t cur2;          // 1: the other operand is a current-event attribute too (no constant)
  int32_t attr2, conv2;  //    (lhs = attr, rhs = attr2)
};

struct RatchetGroup {
  int32_t n_lanes;
  int32_t stream;
  int32_t key_attr, key_conv, key_kind;   // x-atom operand column (same on both sides)
  int32_t xmask;                          // normalized `cur OP key` CmpMask (never EQ/NE)
  int32_t n_f0;
  int32_t sum_slot;                       // row of the launch's per-tile x-summaries (host-set)
  int32_t sim;                            // the SIM kernel form applies (nfa_ratchet.hip; host-set)
  int32_t cell;                           // direct placement: the group's position among its stream's
                                          //   groups in receiver-rank order (host-set; -1: none)
  int32_t pad_cell;
  RatchetAtom f0[RMAXF0];
  int64_t wmax;                           // max within over lanes (-1: none)
  int32_t qid[64];
  int64_t within[64];                     // per lane; INT64_MAX = none
  int64_t f0c[RMAXF0][64];                // per lane constant key of each f0 atom
  // K_gate (nfa_gate.hip): e2's event-only conjuncts `g` (constant atoms, per-lane constants as f0's);
  // n_g > 0 makes the group gated
  int32_t n_g;
  int32_t pad_g;
  RatchetAtom g[RMAXF0];
  int64_t gc[RMAXF0][64];
};

struct RatchetItem {
  int32_t g;          // group
  int32_t chunk, n_chunks;
  int32_t inb;        // state buffer holding the group's current deques
  int64_t c0, c1;     // events this item emits for
};

// persisted per-group deque state: n[64] + entries [rsmax][64] x {ts0, seq, key}
struct RatchetState {
  int32_t n[64];
  int32_t pad[64];
};

struct RatchetLaunch {
  const RatchetGroup* groups;
  const RatchetItem* items;
  int32_t n_items;
  int32_t full_expiry;          // timestamps seen out of order: scan the whole deque for expiry
  StreamBatch b;
  RatchetState* st[2];          // [g]
  int64_t* ent_ts[2];           // [g][rsmax][64] ts0
  int64_t* ent_seq[2];          // [g][rsmax][64] e1 sequence number
  int64_t* ent_key[2];          // [g][rsmax][64] key (32-bit kinds in the low word)
  int64_t rsmax;                // persisted entries per lane (>= ML + SC)
  const uint64_t* tsum_max;     // [slot][n_tiles] max / min key of the valid x of each aligned
  const uint64_t* tsum_min;     //   64-event tile (warm-up skips tiles that cannot hold a survivor)
  const uint8_t* tsum_has;      //   tile has a valid x
  int64_t n_tiles;
  int64_t* lds_ts;              // [item][ML][64] ts0 of the LDS ring entries
  uint4* spillA;                // [item][SC][64] deque entries beyond the LDS ring
  uint32_t* spillB;             //   (seq words of 64-bit-key entries)
  // match records, in per-wave blocks of blk_recs * 8 bytes (16 B per record when wide; the block's
  // group is blk_group[block], its record count blk_count[block]; include/siddhi_hip.h sdh_records
  // documents the formats for consumers). Narrow (wide == 0, batches of at most 2^26 events): 8 B
  // {e2 batch offset | lane << 26, low 32 bits of e1's seq}; wide: 16 B {e2 batch offset, lane, low
  // 32 bits of e1's seq, pop level (placement) or 0}. A wave takes its blocks with an atomic on
  // blk_next; past n_blocks it writes into the spare block, sets err[2], and the host re-runs the push
  // with blk_next's final count of blocks (blocks never wrap)
  int64_t* match;
  int32_t* blk_count;           // records written per block
  int32_t* blk_group;           // group of the wave that owns the block
  int32_t* blk_next;            // [0] next free block
  int32_t n_blocks, blk_recs;
  int32_t wide;
  int32_t dev_records;          // SDH_FLAG_DEVICE_MATCHES: records stay on the device for a consumer
                                //   (sdh_engine_poll_records); rec_total[0] counts them, [2] their bytes
  // rec4 (device records, SIM form, batches of at most 2^26 events): 4-B entries {e1 distance back
  // from e2 (< 2^26) | lane << 26} from the block's start, and per matching event one side entry
  // {index of the event's first entry, e2 batch offset} (uint2) from the block's end downwards (side
  // entry j at byte blk_recs * 8 - 8 * (j + 1); blk_side[block] counts them). A distance >= 2^26
  // sets err[4]; the host then re-runs with 8-B records
  int32_t rec4;
  int32_t* blk_side;
  unsigned long long* rec_total;
  int32_t* err;                 // [0] deque overflow, [1] unordered ts, [2] match overflow, [3] aged,
                                //   [4] a rec4 distance past 2^26
  // direct R18 placement, two passes over the same items (nfa_ratchet.hip PM; the stream's groups
  // hold consecutive receiver ranks in lane order, groups in `cell` order): COUNT stores each
  // (event, group) match total at pcnt[event * n_cells + cell]; WRITE reads their exclusive scan
  // (pbase, same layout) and writes every match as its compact row (cw int32: query, e2 - seq_ref,
  // e2 - e1, 0, INT32_MIN...) at row row0 + pbase[cell] + the lane's rank-ordered offset + its
  // count - 1 - pop level (R18: per event by rank, per query oldest partial first)
  int32_t* pcnt;
  const int32_t* pbase;
  int32_t* crow;
  int64_t row0, seq_ref;
  int32_t n_cells, cw;
};

// ------------------------------------------------------------------------------------------
// K_gen launch (nfa_gen.hip): item = (segment of one key's events, group of 64 queries)
// ------------------------------------------------------------------------------------------
namespace kg {
struct GQuery;
}

// the longest K_gen match record (7 + S + pool nodes words); the flat record buffer is at least twice it
constexpr int64_t GEN_RING_MARGIN = 8192;

struct GenLaunch {
  const kg::GQuery* queries;
  const int32_t* lane_q;      // [group][64] query index (-1 = idle lane)
  const int32_t* group_tmpl;  // [group] query whose structure every lane of the group shares
  StreamBatch b;
  const int32_t* seg_begin;   // [n_seg] ranges into ev_idx (nullptr: one segment = whole batch)
  const int32_t* seg_len;
  const uint32_t* seg_kid;    // dense key id per segment (0xFFFFFFFF: dropped events)
  const int64_t* key_of_id;   // raw key per dense id (nullptr: unpartitioned, key -1)
  const int32_t* ev_idx;      // event indices grouped by key (nullptr: identity)
  int32_t groups;             // groups per segment
  int32_t group_base;         // first row of lane_q for this launch
  int64_t block_base;         // arena block of (kid, g) = block_base + kid * groups + g
  int32_t* a32;
  int64_t* a64;
  int32_t B32, B64;           // arena words per lane and block
  int32_t hot_s, hot_nu;      // LDS hot-word cache extents: max states, max node-mask words
  int64_t* out;               // flat record words: [len, qid, key, ts, seq, idx, S, (count, seqs...)xS]...
  int64_t out_cap;            // words
  unsigned long long* out_next;  // words used (atomic; may run past out_cap on overflow)
  int32_t n_items;
  int32_t* err;               // [0] instance capacity, [1] reference would throw, [2] output overflow
  unsigned long long* rec_count;  // matches emitted (records), counted even when not written
  int64_t* rec_off;           // write_records == 1: word offset of each record, in reservation order
  int64_t rec_cap;
  unsigned long long* rec_next;
  int32_t write_records;      // 1: write; 2: write into a ring nobody reads (SDH_FLAG_DEVICE_MATCHES); 0: count only
  // event chunks of an unpartitioned set (kg::seq_lookback): item = chunk * groups + g; chunk 0
  // continues the persistent arena, chunk c > 0 starts a fresh instance in scratch block
  // (c-1) * groups + g and replays the template's look-back events before emitting
  const int32_t* glist;       // unpartitioned: the set-relative groups this launch runs (item % n_glist)
  int32_t n_glist;
  int32_t ev_chunks;          // 1: unchunked
  int64_t chunk_len;
  int32_t* s32;               // scratch arenas of chunks 1 .. ev_chunks-1
  int64_t* s64;
  // absent states (kgen.h fire_timers): the runtime's start time (instances seeded now schedule
  // their start checks from it), timers due up to each event fire before it, and after the last
  // event those due up to advance_to (INT64_MIN: none; a time advance with no events)
  int64_t start_ts;
  int64_t advance_to;
  int64_t timer_seq;          // trigger seq of the timers fired after the last event
  int32_t playback;           // @app:playback: the generator's time is the event time while timers fire
  int32_t no_timers;          // a chunk push: its timers fired before it (time moved once), none inside
  int32_t xcd;                // items in per-XCD ranges (as PartLaunch)
  // indexed timer sweep (pm != nullptr; batches with ordered timestamps): item = (kid, group) over
  // every known key walks only its own events (the routed segment kseg[kid] of seg_begin / seg_len /
  // ev_idx, -1: none) and fires each due timer at the first batch event whose ts reaches it (binary
  // search in the prefix max pm) -- O(own events + firings) instead of O(batch) per key
  const int64_t* pm;          // [n] prefix max of the batch timestamps
  const int32_t* kseg;        // [known keys] segment of the key's events in this batch, or -1
  // timer sweep of a partition set with absent states: item = (kid, group) over every known key; the
  // item walks the whole batch in order, firing the clone's timers before each event and processing
  // the events of its own key (ev_kid: each event's dense key id); clones seed at their first event
  int32_t sweep;
  const uint32_t* ev_kid;
  int64_t n_keys;
  // fan-out (a stream the partition does not key; with sweep): every event is every key's own; a
  // match record's idx word carries the key's position in the reference's junction map
  // (chm_order.h) above the emission index: fan_pos[kid] << 32 | idx
  const int32_t* fan_pos;
};

// ------------------------------------------------------------------------------------------
// K_part launch (nfa_part.hip): shape-specialised partitioned patterns on compact partial tables
//   PK_OR / PK_AND:  every e1=S[f1] -> e2=S[f2] or|and e3=S[f3] [within T]
//   PK_COUNT:        every e1=S[f1] -> e2=S[f2] <min:max> -> e3=S[f3(e1, e2[0], e2[last], cur)] [within T]
// item = (segment of one key's events, group of 64 same-shape queries); state block of (key, group)
// = [header words][cap entries x entry words], every word lane-interleaved ([word][lane], int64),
// double-buffered across pushes so a push can be re-run exactly with a larger `cap`.
// ------------------------------------------------------------------------------------------
enum PartKind { PK_OR = 0, PK_AND = 1, PK_COUNT = 2 };
constexpr int PK_HDR = 2;      // header words: n entries; logical: filled prefix F | side << 32
constexpr int PK_CMAX = 8;     // count <min:max> with max <= PK_CMAX on K_part
// count-kind entry words: ts1, seq1, flags (len | inL3 << 8 | null bits << 16), chain[max], then
// the captured words the e3 filter reads: e1's, the chain's first event's, its last event's

// K_part's narrow match record (int64 words; beside K_gen-format records in the same buffer -- a
// K_gen record's first word is its positive length, a narrow one's low half is minus its length):
//   w0 = (uint32)(-words) | qid << 32
//   w1 = (uint32)(trigger seq - the batch's seq_base) | key id << 32
//   then int32 seq distances back from the trigger, two per word:
//     PK_OR / PK_AND: e1, side A, side B (INT32_MIN: the side is empty), pad      -> 4 words (32 B)
//     PK_COUNT:       e1, chain length c, the chain's c events (e3 is the trigger) -> 3 + ceil(c / 2)
// The table append (matches.hip) restores the K_gen row: ts from the batch, the key from the
// partition's key table, emission index = e1's seq (the pending-list order is the creation order).
// A match whose distances do not fit int32 goes out as a K_gen record instead.
// K_seq's narrow record (kind 2 in w0's low half: -(words + 0x20000)), an unpartitioned window match:
//   w0 = (uint32)(-(words + 0x20000)) | qid << 32
//   w1 = (uint32)(trigger seq - the batch's seq_base) | S << 32
//   then the S - 1 earlier slots' int32 seq distances back from the trigger, two per word
//                                                                        -> 2 + S / 2 words (24 B at S = 3)
// restored as [(1, seq) x S] with key -1, ts from the batch, emission index 0 (one match per event
// and query).
constexpr int NREC_ORAND_WORDS = 4;
constexpr int NREC_KIND_COUNT = 1, NREC_KIND_SEQ = 2;
__host__ __device__ inline int nrec_count_words(int c) { return 3 + (c + 1) / 2; }
__host__ __device__ inline int nrec_seq_words(int S) { return 2 + S / 2; }
constexpr int NREC_MIN_WORDS = 3;  // (K_seq's at S <= 3; record-offset capacities are words / 3)
__host__ __device__ inline int64_t nrec_pack(int64_t lo, int64_t hi) {
  return (int64_t)(((uint64_t)(uint32_t)(int32_t)lo) | ((uint64_t)(uint32_t)(int32_t)hi << 32));
}

struct PartLaunch {
  const kg::GQuery* queries;
  const int32_t* lane_q;      // [group][64]
  const int32_t* group_tmpl;  // [group]
  StreamBatch b;
  const int32_t* seg_begin;   // partition routing (as GenLaunch)
  const int32_t* seg_len;
  const uint32_t* seg_kid;
  const int64_t* key_of_id;
  const int32_t* ev_idx;
  int32_t groups;             // groups of this set; state block (kid, g) = kid * groups + g
  int32_t group_base;         // first row of lane_q / group_tmpl of the set
  int32_t kind;               // PartKind
  int32_t cap;                // entries per lane
  int32_t ew;                 // words per entry
  int32_t g0, gn;             // this launch runs groups g0 .. g0+gn-1 of the set (one shape)
  int32_t sA, sB;             // logical: state ids of the side processed second (A) and first (B)
  int32_t cmax;               // count: chain words per entry (the set's largest max)
  int32_t n_e1, n_first, n_last;  // count: captured words stored per entry (0 or the stream's n_cap)
  int32_t n_items;            // key segments x gn
  int64_t* st;                // [buffer 0/1][block][PK_HDR + cap * ew][64], block = kid * groups + g
  int64_t blocks;             // blocks per buffer
  const int32_t* cur;         // [kid] buffer holding the key's tables before this push
  int32_t* nxt;               // [kid] after it (the host swaps cur / nxt once the push succeeded)
  int64_t* out;               // K_gen-format match records (nfa_gen.hip), as GenLaunch
  int64_t out_cap;
  unsigned long long* out_next;
  unsigned long long* rec_count;
  int64_t* rec_off;
  int64_t rec_cap;
  unsigned long long* rec_next;
  int32_t write_records;
  int32_t xcd;                // items in per-XCD ranges (dev::grid_item; the grid is padded to a multiple of 8)
  int32_t sorted;             // b holds the batch in key order (position t = ev_idx's t); ev_idx still
                              // gives each position's batch index (its seq)
  int32_t* err;               // [0] entry capacity, [2] output overflow
  unsigned long long* prof;   // SDH_PART_PROF builds: per-phase clock sums (part_body.h), else null
  const int64_t* lconst;      // [group][lc_slots][64] the lanes' query ids, withins, constants (kg::LaneConsts)
  int32_t lc_slots;
  int32_t pad_lc;
};

// ------------------------------------------------------------------------------------------
// K_slab launch (nfa_slab.hip): distinct-stream patterns on sparse per-partial entries (slab.h)
// item = (key segment of the pushed stream, group from glist); block (kid, g) = dir[kid * groups + g]
// in sub-ring sub_of(kid * groups + g) (a separately allocated ring buffer)
//   dir word: offset / 4 in the sub-ring (bits 0-31) | entries (40-55) | states with a non-empty list (56-63)
// ------------------------------------------------------------------------------------------
namespace slab {
struct Shape;
}

struct SlabLaunch {
  const kg::GQuery* queries;
  const int32_t* lane_q;      // [group][64]
  const int32_t* group_tmpl;  // [group]
  const slab::Shape* shapes;  // per shape
  const int32_t* group_shape; // [set group] -> shape
  StreamBatch b;
  const int32_t* seg_begin;   // partition routing (as GenLaunch)
  const int32_t* seg_len;
  const uint32_t* seg_kid;
  const int64_t* key_of_id;
  const int32_t* ev_idx;
  const int32_t* glist;       // set groups that read the pushed stream; item = seg * n_glist + j
  int32_t n_glist;
  int32_t n_items;
  int32_t groups;             // groups of the set (directory stride)
  int32_t group_base;         // first row of lane_q / group_tmpl of the set
  uint64_t* dir;              // [key_cap * groups]
  uint64_t* journal;          // [item] the directory value a changed item replaced
  uint64_t* journal_idx;      // [item] its directory index (~0: unchanged; the host clears them)
  uint32_t* const* ring;      // [nsub] sub-ring buffers
  const int64_t* ring_cap;    // [nsub] words of each
  unsigned long long* head;   // [nsub] logical allocation heads (monotone)
  const unsigned long long* tail;  // [nsub] oldest live logical word
  int32_t nsub;
  int32_t lds_words;          // dynamic LDS (uint32 words) for a block's entries
  int32_t max_na;             // the widest captured-word count of the set's shapes (event staging)
  long long* live;            // [256] live-partial counters (sum = live partials)
  unsigned long long* traffic;  // [256] block bytes read + written (the launch's state traffic)
  int64_t* out;               // K_gen-format match records, as GenLaunch
  int64_t out_cap;
  unsigned long long* out_next;
  unsigned long long* rec_count;
  int64_t* rec_off;
  int64_t rec_cap;
  unsigned long long* rec_next;
  int32_t write_records;
  int32_t xcd;                // items in per-XCD ranges (as PartLaunch)
  int32_t* err;               // [0] LDS capacity, [1] slab space, [2] output overflow
  const int64_t* lconst;      // [group][lc_slots][64] the lanes' query ids, withins, constants (kg::LaneConsts)
  int32_t lc_slots;
  int32_t defer_cap;          // two-tier LDS: room in defer (0: no deferral, an oversized block sets err[0])
  int32_t* defer;             // items whose block outgrew this launch's LDS rows (re-run with more LDS)
  int32_t* defer_n;
  const int32_t* item_list;   // the deferred launch: its items (nullptr: items 0 .. n_items-1)
};

// ------------------------------------------------------------------------------------------
// K_seq launch (nfa_gen.hip): every-start single-stream sequences of stream states evaluated as
// windows of S consecutive events (kg::seq_window); item = (start chunk, group of 64 queries)
// ------------------------------------------------------------------------------------------
constexpr int SEQ_TMAX = 7;                   // events a stream's tail carries (GMAXS - 1)
constexpr int SEQ_TW = 2 + 2 * MAXATTR;       // tail row: ts, seq, raw words, null flags

struct SeqLaunch {
  const kg::GQuery* queries;
  const int32_t* lane_q;      // [group][64] query index (-1 = idle lane)
  const int32_t* group_tmpl;  // [group] shape template
  const int32_t* glist;       // [n_glist] groups (rows of lane_q) this launch runs
  int32_t n_glist;
  int32_t n_chunks;           // start chunks per group
  int64_t chunk_len;          // window starts per chunk
  StreamBatch b;
  const int64_t* tail;        // [SEQ_TMAX][SEQ_TW]: the stream's last events before this batch
  int32_t tail_len;
  int32_t write_records;
  int64_t* out;               // flat K_gen-format records (nfa_gen.hip)
  int64_t out_cap;
  unsigned long long* out_next;
  unsigned long long* rec_count;
  int64_t* rec_off;           // as GenLaunch
  int64_t rec_cap;
  unsigned long long* rec_next;
  int32_t* err;               // [2] output overflow
  int32_t xcd;                // items in per-XCD ranges (as PartLaunch)
};

// ------------------------------------------------------------------------------------------
// Device match table (matches.hip): every plan's matches since the last poll, one row each, with
// the R18 delivery-order sort keys (the reference hands each completed StateEvent to
// QuerySelector.process per input event, per receiver, per state processor, per pending partial):
//   hi    = (trigger seq - seq_ref) << RANK_BITS | out_rank(query, stream)
//   lo[k] = tiebreaks of one (trigger event, query), least significant first: K_ratchet the e1
//           seq; K_chain slot k's seq (k = 0 .. S-2; slot S-2 is compared first); K_gen the
//           emission index within its processAndReturn chunk
// words[woff .. woff+wlen) = per state slot a count c then c event sequence numbers.
// A poll window holding chunk pushes (sdh_batch.chunk) sorts by two more significant keys first:
//   chi = (chunk's first seq - seq_ref) << RANK_BITS | junction subscriber rank
//   clo = (same-key run start | fan-out key position) << RANK_BITS | the query's rank in its partition
// (single-event rows and timer rows: chi = their hi with rank 0, clo = 0; matches.hip chunk_keys).
// ------------------------------------------------------------------------------------------
constexpr int MAXLO = MAXS - 1;
constexpr int RANK_BITS = 20;

struct MatchTable {
  uint64_t* hi;
  uint64_t* lo[MAXLO];
  uint64_t* chi;
  uint64_t* clo;
  int64_t* seq;         // trigger event sequence number
  int64_t* q;
  int64_t* key;
  int64_t* ts;
  int64_t* woff;
  int64_t* wlen;
  int64_t* words;
};

}  // namespace sdh
