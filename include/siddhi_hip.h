/*
 * siddhi_hip.h -- C-ABI of libsiddhi_hip.so, the MI355X pattern/sequence (NFA) engine.
 *
 * This is the drop-in boundary for the reference's state-stream path
 * (org.wso2.siddhi.core.query.input.stream.state). Each entry point replaces one seam of the
 * reference (paths relative to modules/siddhi-core/src/main/java/org/wso2/siddhi/core/):
 *
 *   sdh_engine_create   <- util/parser/InputStreamParser.java:94-99 (state branch) +
 *                          util/parser/StateInputStreamParser.java:77-143 (parseInputStream) +
 *                          query/QueryRuntime.java:186-193 (init: seeds the start states)
 *   sdh_engine_push     <- stream/StreamJunction.java:376-389 (Receiver.receive(Event[]) /
 *                          receive(long, Object[])) -> query/input/ProcessStreamReceiver.java:105-183
 *                          -> state/StreamPreStateProcessor.java:292-337 (processAndReturn)
 *   sdh_engine_poll     <- query/input/SingleProcessStreamReceiver.java:75-79 and
 *                          query/input/StateMultiProcessStreamReceiver.java:65-72 (hand-off of each
 *                          completed StateEvent to QuerySelector.process)
 *   sdh_engine_poll_device  the same matches left in HBM (device consumers of the matches)
 *   sdh_engine_poll_compact the same matches as 16-B compact rows (host or HBM)
 *   sdh_engine_poll_compact_ex  every match as compact rows + key ids, timer tiebreaks and count
 *                          chains (the StateEvent contents of StateEvent.java:138-182)
 *   sdh_engine_poll_records the matches as the kernels wrote them, left in HBM for a device consumer
 *                          (SDH_FLAG_DEVICE_MATCHES; the formats are documented below)
 *   sdh_engine_set_strings  <- partition/PartitionStreamReceiver.java:277-281 (String.valueOf of a
 *                          string key: its hashCode / length, for the fan-out order)
 *   sdh_engine_reserve / sdh_engine_reserve_keys
 *                       <- partition/PartitionRuntime.java:257-306 (per-key clones created lazily):
 *                          state sized up front, so no push stalls on growth
 *   sdh_comm_* / sdh_engine_set_comm / sdh_engine_push_bcast / sdh_engine_gather
 *                       <- stream/StreamJunction.java:179-181 (every subscriber of a junction) when the
 *                          subscribers are sharded over the GPUs of a node: RCCL broadcast of each
 *                          batch, gather + device k-way merge of the matches in R18 order
 *   sdh_engine_flush    <- (no reference equivalent: the reference is synchronous)
 *   sdh_engine_snapshot / sdh_engine_restore
 *                       <- state/StreamPreStateProcessor.java:352-367 (currentState/restoreState)
 *   sdh_last_error      <- Java exceptions (SiddhiAppCreationException, OperationNotSupportedException)
 *
 * Conventions: plain C, no exceptions cross the ABI, every call returns 0 on success and a
 * negative SDH_E* code on failure; sdh_last_error() then describes it. Capacity overflows inside a
 * push (pools, lists, tables, slab rings, match output) grow the buffer and re-run the push exactly
 * from a journal, so no push drops a match. A push that fails after its kernels ran (device memory
 * exhausted while growing, a HIP error, SDH_E_REFERENCE) leaves the engine unusable: later calls
 * fail with SDH_E_CAPACITY until sdh_engine_restore. One producer thread per
 * engine (the reference serialises receivers on a monitor, SingleProcessStreamReceiver.java:59).
 * There is NO CPU fallback: an engine that cannot run a query on the GPU fails at create time.
 */
#ifndef SIDDHI_HIP_H
#define SIDDHI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDH_OK 0
#define SDH_E_INVALID (-1)     /* bad argument / malformed IR                               */
#define SDH_E_UNSUPPORTED (-2) /* query shape not executable on the GPU path                */
#define SDH_E_DEVICE (-3)      /* HIP runtime error                                          */
#define SDH_E_CAPACITY (-4)    /* a partial-match table or match buffer overflowed (see below) */
#define SDH_E_REFERENCE (-5)   /* the reference engine would throw here (e.g. CME)           */

typedef struct sdh_engine sdh_engine;

typedef struct sdh_config {
  int32_t device;            /* HIP device ordinal (one process per GPU)                      */
  int32_t shard_rank;        /* multi-GPU: an unpartitioned query q runs here iff             */
  int32_t shard_world;       /*   q % shard_world == shard_rank (1/0 = unsharded); partitioned */
                             /*   queries run on every rank for the keys this rank owns:       */
                             /*   |String.valueOf(key).hashCode() % shard_world| == shard_rank */
                             /*   (PartitionedDistributionStrategy.java:98-109)                */
  int32_t partials_per_inst; /* live partial-match capacity per query instance (mult. of 64) */
  int64_t max_batch;         /* max events per push                                          */
  int64_t match_capacity;    /* max matches held between polls (0 = sized automatically)     */
  int32_t chunk_events;      /* target events per parallel chunk (0 = automatic)             */
  int32_t flags;             /* SDH_FLAG_*                                                   */
  /* K_gen (general interpreter) pools per query instance (0 = defaults 64 / 128 / 48) and the
   * partition key capacity (0 = 2^20 keys per partition). These are starting sizes: a push that
   * overflows a pool or list is undone, the pools double (up to 4096 StateEvents / nodes) and the
   * push is re-run exactly (sdh_stats.pool_regrows).                                         */
  int32_t gen_pool_states;   /* StateEvent objects (<= 4096)                                 */
  int32_t gen_pool_nodes;    /* chained event copies (<= 4096)                               */
  int32_t gen_list_cap;      /* entries per pending / newAndEvery list                       */
  int32_t gen_pad;
  int64_t gen_max_keys;      /* distinct partition keys per partition                        */
  /* Tuning / diagnostic overrides, "NAME=VALUE;NAME=VALUE" (NULL: none), copied at create: kernel
   * A/B knobs, traces, and test hooks that force a code path (DESIGN.md §8 lists them). The library
   * reads no environment variables, so a host process's environment never changes its behaviour. */
  const char* debug;
} sdh_config;

/* Device records: a push leaves its matches in HBM as the kernels wrote them (no R18 sort, no
 * match table), for consumers on the device: sdh_engine_poll_records hands them out (formats below),
 * valid until the next push. Every match of the push is written (the record buffers grow and the push
 * re-runs exactly, as in the normal mode); a push's records that nobody reads are dropped at the next
 * push (sdh_engine_pending_matches counts them until then). sdh_engine_poll and the compact polls
 * return nothing in this mode. */
#define SDH_FLAG_DEVICE_MATCHES 1
/* Disable the K_ratchet plan (every query of that shape runs on the general chain kernel instead);
 * for differential testing of the two plans. */
#define SDH_FLAG_NO_RATCHET 2
/* Run every query on the general interpreter K_gen (no chain / ratchet plans); for differential
 * testing. */
#define SDH_FLAG_FORCE_GEN 4
/* @app:playback: while absent states' timers fire, the runtime's time is the event time that let
 * them fire (TimestampGeneratorImpl.currentTime in playback), not the timer's own time. */
#define SDH_FLAG_PLAYBACK 8

/* One columnar (SoA) batch of events of one stream, in arrival order.
 * cols[a] points to n elements of attribute a with the stream schema's native width:
 *   INT -> int32, LONG -> int64, FLOAT -> float, DOUBLE -> double, BOOL -> uint8,
 *   STRING -> int32 dictionary id (ids are assigned by the caller; equal strings, equal ids).
 * nulls[a] (optional, may be NULL or have NULL entries) is a uint8 mask, 1 = null.
 * on_device != 0: all pointers are HIP device pointers already resident in HBM, and their contents
 * complete (the engine runs on its own non-blocking stream: the caller synchronizes the stream that
 * produced them); otherwise they are host pointers (pinned memory recommended) and are copied before
 * sdh_engine_push returns.
 * chunk != 0: the batch is ONE chunk, InputHandler.send(Event[]) (stream/input/InputHandler.java:77-85)
 * -> StreamJunction.sendEvent(Event[]) (stream/StreamJunction.java:218-236): every junction
 * subscriber (a query, or a partition) receives the whole chunk before the next one; a partition
 * splits it into runs of consecutive same-key events, each run going to its key's clones in turn
 * (partition/PartitionStreamReceiver.java:214-239), or sends all of it to every key for a stream it
 * does not key (:200-213, 277-281); a single-stream receiver calls its selector at the end of its
 * chunk (query/input/SingleProcessStreamReceiver.java:57-80). Time moves once, to the chunk's last
 * timestamp, before the chunk: the absent states' timers due by then fire first, none inside it.
 * chunk == 0: n single-event sends (InputHandler.send(Event) per event). */
typedef struct sdh_batch {
  int64_t n;
  const int64_t* ts;
  const void* const* cols;
  const uint8_t* const* nulls;
  int32_t n_cols;
  int32_t on_device;
  int32_t chunk;
  int32_t reserved;          /* 0 */
} sdh_batch;

/* Matches, in the reference's delivery order (per input event; per query; per state processor
 * in reverse registration order; per pending partial in insertion order -- SURVEY R18; for a chunk
 * push: per junction subscriber, per same-key run or key, per query, per event, ...). The
 * order is established on the device (a stable radix sort of the matches since the last poll).
 * Match i: query[i], key[i] (partition key id, -1 if unpartitioned), ts[i] (the StateEvent
 * timestamp); words[off[i] .. off[i+1]) holds, per state slot, a count c followed by c global
 * event sequence numbers (the slot's event chain when the selector would have run).
 * seq[i] is the sequence number of the event whose processing completed the match (the R18 order
 * is by that event first; a multi-GPU gather merges per-rank outputs on it).
 * Sequence numbers count pushed events from 0 across all streams in push order.
 * tb[i] is INT64_MIN for a match completed by an event; for an absent state's timer match (fired
 * before event seq[i], or by sdh_engine_advance_time) it is the instance's running max of the times
 * fired so far: the timer matches of one seq precede its event matches, ordered by (tb, query, key)
 * and then by emission (the order a multi-GPU merge needs, siddhi_amd/dist.py).
 * Buffers are owned by the engine and valid until the next push/poll/destroy. */
typedef struct sdh_matches {
  int64_t n;
  const int64_t* query;
  const int64_t* key;
  const int64_t* ts;
  const int64_t* off;
  const int64_t* words;
  const int64_t* seq;
  const int64_t* tb;
} sdh_matches;

typedef struct sdh_stats {
  int64_t events;            /* events pushed                                                */
  int64_t pattern_events;    /* sum over pushes of events x queries consuming that stream    */
  int64_t matches;           /* matches produced                                             */
  int64_t live_partials;     /* live partial matches after the last push                     */
  double last_kernel_ms;     /* device time of the last NFA-step launch (HIP events)         */
  double last_kernel_bytes;  /* algorithmic bytes of that launch (DESIGN.md roofline model)   */
  int64_t last_gen_items;    /* K_gen work items (waves) of the last push: groups x key       */
                             /* segments, or groups x event chunks           */
  int64_t last_seq_items;    /* K_seq work items of the last push: groups x window chunks     */
  int64_t last_part_items;   /* K_part work items of the last push: groups x key segments     */
  double last_ingest_ms;     /* host-to-HBM copy time of the last host-resident batch (side   */
                             /* stream; 0 for on_device batches)                              */
  int64_t ingest_bytes;      /* bytes copied from host batches so far                         */
  int64_t spec_kernels;      /* shape-compiled kernels this engine launches (hiprtc at create; */
                             /* SDH_SPEC=0 off, 1 every shape, default shapes of >= 128 queries) */
  int64_t pool_regrows;      /* K_gen pool / list growths (each re-lays the arenas and re-runs   */
                             /* the push that overflowed; the reference's lists are unbounded)   */
  int64_t last_slab_items;   /* K_slab work items of the last push: key segments x groups         */
  int64_t placed_pushes;     /* pushes whose matches (all K_ratchet) went straight to their R18   */
                             /* rows (no sort at poll; matches.hip ratchet_place_kernel)          */
  int64_t plan_queries[8];   /* queries (pattern instances of this shard) per device plan:         */
                             /* [0] K_ratchet [1] K_gate [2] K_chain [3] K_part [4] K_slab         */
                             /* [5] K_seq [6] K_gen                                */
} sdh_stats;

int sdh_engine_create(const void* ir_blob, size_t len, const sdh_config* cfg, sdh_engine** out);
int sdh_engine_push(sdh_engine* e, int32_t stream, const sdh_batch* batch);
int sdh_engine_flush(sdh_engine* e);
int sdh_engine_poll(sdh_engine* e, sdh_matches* out);
/* As sdh_engine_poll, but every sdh_matches pointer is a HIP device pointer into engine-owned HBM
 * (valid until the next push/poll/destroy): no copy to the host. */
int sdh_engine_poll_device(sdh_engine* e, sdh_matches* out);
/* The same matches in the same order as compact int32 rows (4 * width bytes per match),
 * for consumers that hold their own events and want the match relation only: row i is
 * rows[i * width .. (i + 1) * width) =
 *   { query, seq_i - seq_base, then per state slot seq_i - the slot's event seq (0 for the event
 *     that completed the match), or INT32_MIN for an empty slot / a slot the query lacks },
 * where seq_i is sdh_matches.seq[i]; width = 2 + the most states any query of the engine has.
 * A window whose matches came straight from K_ratchet placement is handed out without a sort or a
 * gather (4 int32 per match instead of 8 int64 + 4 words). Matches this form cannot express (a slot
 * holding a chain of several events -- count states --, a partition key, an absent state's timer
 * match, seq distances past 2^31) fail with SDH_E_UNSUPPORTED and stay pending: poll them with
 * sdh_engine_poll. device != 0 leaves rows in engine-owned HBM (valid until the next
 * push/poll/destroy); otherwise they are copied to an engine-owned host buffer. */
typedef struct sdh_matches_compact {
  int64_t n;
  int64_t seq_base;
  int32_t width;
  int32_t flags;             /* 0 */
  const int32_t* rows;
} sdh_matches_compact;
int sdh_engine_poll_compact(sdh_engine* e, int32_t device, sdh_matches_compact* out);
/* Compact rows for every match (count-state chains, partition keys and absent-state timer matches
 * included: StateEvent.getStreamEvent:138-182 resolves a count slot to its chain; the key is
 * PartitionStreamReceiver.java:270-275's per-key delivery). Row i is rows[i * width .. (i + 1) * width):
 *   { query, seq_i - seq_base, then per state slot v: v >= 0 one event (seq_i - its seq),
 *     INT32_MIN an empty slot, v < 0 a chain: chain[-(v + 1)] = its event count c, followed by the c
 *     distances seq_i - seq (a count slot with one event is a plain distance) },
 * key[i] the partition key (as sdh_matches.key; NULL when no query is partitioned), tb[i] the timer
 * tiebreak (as sdh_matches.tb; NULL when no query has absent states). Only seq distances past 2^31
 * fail (SDH_E_UNSUPPORTED, the matches stay pending). device != 0: engine-owned HBM. */
typedef struct sdh_matches_compact_ex {
  int64_t n;
  int64_t seq_base;
  int32_t width;
  int32_t flags;             /* 0 */
  const int32_t* rows;
  const int64_t* key;
  const int64_t* tb;
  int64_t n_chain;           /* int32 words in chain */
  const int32_t* chain;
} sdh_matches_compact_ex;
int sdh_engine_poll_compact_ex(sdh_engine* e, int32_t device, sdh_matches_compact_ex* out);
/* Device-resident match count of the last push (no host copy of the matches). */
int sdh_engine_pending_matches(sdh_engine* e, int64_t* n);
/* ---- Device records (SDH_FLAG_DEVICE_MATCHES) ----
 * The last push's matches as the kernels wrote them, in three parts; every pointer is a HIP device
 * pointer into engine-owned HBM, valid until the next push/restore/destroy. Records are in no
 * particular order (wave completion order); a consumer that needs the reference's delivery order
 * sorts them by (trigger seq, receiver rank, ...) -- or polls in the normal mode. Sequence numbers:
 * the push's event at batch offset k has seq seq_base + k (sdh_matches.seq). The call also marks the
 * records consumed (sdh_engine_pending_matches returns 0 until the next push).
 *
 * 1. K_ratchet blocks (the `every e1=S[f] -> e2=S[cur.a OP e1.a] within T` plan: DESIGN.md §3.1).
 *    Block b (0 <= b < r_blocks) is r_blk_bytes at (const char*)r_base + b * r_blk_bytes and belongs
 *    to wave group g = r_group[b]; a record's lane l names query r_lane_query[g * 64 + l]. It holds
 *    r_count[b] records of format r_format:
 *      SDH_REC_8:  uint32 pairs {e2 | l << 26, e1lo}: e2 = the trigger's batch offset (bits 0-25),
 *                  e1lo = the low 32 bits of e1's seq (e1 = s2 - (uint32)((uint32)s2 - e1lo), s2 =
 *                  seq_base + e2);
 *      SDH_REC_16: uint32 quads {e2, l, e1lo, 0} (batches of more than 2^26 events);
 *      SDH_REC_4:  uint32 entries {d | l << 26} from the block's start, d = s2 - e1 (< 2^26), plus
 *                  r_side[b] side entries, uint32 pairs {first, e2}, from the block's END downwards:
 *                  side entry j at r_blk_bytes - 8 * (j + 1). Entry i belongs to the trigger e2 of the
 *                  last side entry whose `first` <= i (side entry 0 has first == 0; `first` ascends).
 *                  (Only float-keyed queries write rec4 blocks: a block with r_side[b] < 0 in such a
 *                  push holds SDH_REC_8 records.)
 *    sdh_engine_records_compact decodes this part into compact rows on the device.
 * 2. Flat records (the K_gen / K_part / K_seq / K_slab plans): f_words int64 words at f_base, a
 *    sequence of records, each identified by the low 32 bits of its first word, lo = (int32)w[0]:
 *      lo >= 0       a full record of lo words: {lo, query, key, ts, trigger seq, emission index,
 *                    S | stream << 16, then per state slot: c, c event seqs} (stream 0xFFFF: an absent
 *                    state's timer match; key -1 when unpartitioned, else the raw partition key);
 *      -lo >> 16 == 0: K_part logical (or / and) match, -lo words (4): w[0] >> 32 = query,
 *                    w[1] = {trigger batch offset (low 32), partition key id (high 32)}, then int32
 *                    distances back from the trigger (s2 - seq): e1, side A, side B (INT32_MIN: empty);
 *      -lo >> 16 == 1: K_part count match, (-lo & 0xFFFF) words: as above, then e1, chain length c and
 *                    the c chain events' distances (two int32 per word, low half first);
 *      -lo >> 16 == 2: K_seq window match, (-lo & 0xFFFF) words: w[0] >> 32 = query, w[1] = {trigger
 *                    batch offset, S}, then the S - 1 earlier slots' int32 distances;
 *      -lo >> 16 == 4: padding of (-lo & 0xFFFF) words (skip it).
 *    A K_part record's key id is a dense id: f_query_keys[query][id] is the raw partition key (the
 *    sdh_matches.key value; f_query_keys[query] is NULL for an unpartitioned query).
 * 3. K_chain segments (the general chain plan): c_items segments, segment i = c_count[i] records of
 *    c_words int64 at c_base + c_off[i] * c_words, each {query, ts, seq_0 .. seq_{S-1}}.
 */
#define SDH_REC_NONE 0
#define SDH_REC_8 1
#define SDH_REC_16 2
#define SDH_REC_4 3
typedef struct sdh_records {
  int64_t n;                  /* matches in all parts                                          */
  int64_t seq_base;           /* seq of the push's batch offset 0                              */
  int64_t n_events;           /* events of the push                                            */
  /* 1. K_ratchet blocks */
  int64_t r_n;                /* matches in this part                                          */
  int64_t r_blocks;
  int64_t r_bytes;            /* bytes of records written (entries + side entries)             */
  const void* r_base;
  const int32_t* r_count;
  const int32_t* r_side;      /* (SDH_REC_4 blocks)                                             */
  const int32_t* r_group;
  const int32_t* r_lane_query;
  int32_t r_format;           /* SDH_REC_*                                                      */
  int32_t r_blk_bytes;
  /* 2. flat records */
  int64_t f_n;
  int64_t f_words;
  const int64_t* f_base;
  const int64_t* const* f_query_keys; /* [queries] device pointers to the key tables (see above)  */
  /* 3. K_chain segments */
  int64_t c_n;
  int64_t c_items;
  int32_t c_words;
  int32_t flags;              /* 0 */
  const int64_t* c_base;
  const int64_t* c_off;
  const int64_t* c_count;
} sdh_records;
int sdh_engine_poll_records(sdh_engine* e, sdh_records* out);
/* Part 1 of the last push's device records decoded into compact rows of `width` int32 (>= 4) in HBM,
 * in block order: { query, e2 - seq_base, e2 - e1, 0, INT32_MIN ... } (the sdh_matches_compact row of
 * a 2-state match). rows == NULL: *n = the row count only; otherwise rows holds cap rows and
 * SDH_E_CAPACITY is returned if the part has more. */
int sdh_engine_records_compact(sdh_engine* e, int32_t* rows, int64_t cap, int32_t width, int64_t* n);
/* Absent patterns (`not S[..] for T`) and time. The runtime starts at t (SiddhiAppRuntime.start:
 * start states with a 'for' time schedule their first check at t + T); without this call it starts
 * with its first event or advance. sdh_engine_advance_time: time passes to t with no event, and
 * every absent state's scheduler fires what falls due (Scheduler.java:186-287); pushes fire the
 * timers due by each event before it. Replaces: the scheduler thread / playback heartbeat. */
int sdh_engine_start(sdh_engine* e, int64_t t);
int sdh_engine_advance_time(sdh_engine* e, int64_t t);
int sdh_engine_stats(sdh_engine* e, sdh_stats* out);
/* The last push's device time and algorithmic bytes (sdh_stats.last_kernel_ms / last_kernel_bytes)
 * without the rest: no device work and no synchronisation (sdh_engine_stats counts the live partials
 * on the device), for per-push instrumentation. */
int sdh_engine_push_stats(sdh_engine* e, double* last_kernel_ms, double* last_kernel_bytes);
/* Device memory of the sparse per-partial state (K_slab: partitioned distinct-stream patterns,
 * state only for instances that hold partials -- PartitionRuntime.java:257-306 clones per key
 * lazily): live entry bytes, reserved slab bytes, directory bytes. */
int sdh_engine_state_bytes(sdh_engine* e, int64_t* live_bytes, int64_t* reserved_bytes, int64_t* dir_bytes);
/* Pre-allocate `bytes` of HBM for that sparse state (split over the engine's K_slab sets), so it grows
 * inside memory the engine already holds: a state that outgrows it takes more in chunks that double.
 * (One large device allocation can stall for seconds; a deployment that knows its state size sizes it
 * once here, before the first push.) No-op for an engine without K_slab sets. */
int sdh_engine_reserve(sdh_engine* e, int64_t bytes);
/* Size every partitioned state (per-key instance blocks of K_gen / K_part, K_slab key directories)
 * for `keys` distinct partition keys now, so that pushes bringing the first `keys` keys never
 * reallocate and copy that state (a push that does stalls for the copy: the p99 of small pushes while
 * keys keep appearing). The reference creates a key's instances lazily on its first event
 * (partition/PartitionRuntime.java:257-306); results are identical either way. `keys` <=
 * sdh_config.gen_max_keys; SDH_E_INVALID beyond it. */
int sdh_engine_reserve_keys(sdh_engine* e, int64_t keys);
/* The text behind string dictionary ids, as String.hashCode and UTF-16 length per id. Needed only by
 * a partition keyed by a string attribute whose queries also read a stream it does not key: that
 * stream reaches every key's junction in the order of a ConcurrentHashMap of "streamId" +
 * String.valueOf(key) (partition/PartitionStreamReceiver.java:277-281), which hashes the key's text.
 * Register every id such a key can take (a later call may add ids) before the push that needs it,
 * and again after sdh_engine_restore; a missing id fails that push with SDH_E_INVALID. */
int sdh_engine_set_strings(sdh_engine* e, int64_t n, const int32_t* ids, const int32_t* java_hash,
                           const int32_t* utf16_len);
int sdh_engine_snapshot(sdh_engine* e, void** blob, size_t* len);
int sdh_engine_restore(sdh_engine* e, const void* blob, size_t len);
void sdh_free(void* p);
void sdh_engine_destroy(sdh_engine* e);
const char* sdh_last_error(sdh_engine* e);
/* ---- Multi-GPU: one engine per GPU, the exchange inside the library ----
 * Every rank runs the same program with sdh_config.shard_rank / shard_world = its rank in the
 * communicator: unpartitioned queries shard by pattern set (q % world), partitions by key
 * (|String.valueOf(key).hashCode() % world|, PartitionedDistributionStrategy.java:98-109). The
 * exchange has two steps and no other collective:
 *   sdh_engine_push_bcast  every rank pushes the same batch, broadcast from `root`'s copy (RCCL over
 *                          xGMI): StreamJunction.sendEvent reaching every subscriber
 *                          (stream/StreamJunction.java:179-181) when the subscribers live on N GPUs;
 *   sdh_engine_gather      every rank's R18-ordered matches since its last poll go to rank 0, which
 *                          merges the runs on the device (a k-way merge: a receiver's matches of one
 *                          event come from one rank, so the runs never tie) into exactly the order a
 *                          single engine would deliver -- the QuerySelector hand-off of sdh_engine_poll.
 * Communicators:
 *   sdh_comm_get_id + sdh_comm_create: RCCL, one process per GPU (ncclGetUniqueId on one rank, the
 *     SDH_COMM_ID_BYTES distributed by the host -- e.g. over the cluster's own control channel -- and
 *     ncclCommInitRank on every rank; collective: every rank calls it).
 *   sdh_comm_create_local: `world` ranks inside this process (engines on one or several devices),
 *     buffers copied device-to-device: the same protocol, for one process driving several engines and
 *     for testing the exchange on one GPU. Its collectives are one-sided and complete in call order,
 *     so its calls must be serialised (one thread, or the caller orders them): a broadcast's root
 *     pushes first and every other rank receives it before the root's next broadcast; a gather's ranks
 *     1..world-1 call first and rank 0 last, and a rank that has deposited its matches is not polled
 *     again until rank 0 has gathered. A call out of this order fails with SDH_E_INVALID. Copies wait
 *     on the depositing rank's stream (HIP events), so the engines may run on different streams.
 * An invalid batch at the root of sdh_engine_push_bcast fails the call on every rank (the root
 * broadcasts an error header). With RCCL every rank receives every rank's gather header and all
 * refuse an out-of-step window before any table is cleared.
 * sdh_engine_set_comm attaches a communicator (not owned; it must outlive the engine's use of it,
 * and its device must be the engine's). Both exchange calls are collective over the communicator's
 * ranks and run on the engine's stream. */
#define SDH_COMM_ID_BYTES 128
#define SDH_MAX_RANKS 64
typedef struct sdh_comm sdh_comm;
int sdh_comm_get_id(void* id, size_t cap);
int sdh_comm_create(const void* id, size_t len, int32_t rank, int32_t world, int32_t device, sdh_comm** out);
int sdh_comm_create_local(int32_t world, const int32_t* devices, sdh_comm** out /* world entries */);
void sdh_comm_destroy(sdh_comm* c);
const char* sdh_comm_last_error(void);   /* this thread's last sdh_comm_* failure */
int sdh_engine_set_comm(sdh_engine* e, sdh_comm* c);
/* As sdh_engine_push on every rank, with the batch taken from `root`'s `batch` (host or device,
 * single events or a chunk); the other ranks pass NULL (or any batch: ignored) and receive it into
 * engine-owned HBM. */
int sdh_engine_push_bcast(sdh_engine* e, int32_t stream, const sdh_batch* batch, int32_t root);
/* Collective poll: rank 0's `out` receives the matches of every rank since their last poll, merged
 * into the single-engine order (the sdh_engine_poll contract; device != 0: HBM pointers as
 * sdh_engine_poll_device), other ranks get n = 0. Requires shard_rank / shard_world equal to the
 * communicator's rank / world, and every rank's poll windows in step (the same pushes since the last
 * gather). */
int sdh_engine_gather(sdh_engine* e, int32_t device, sdh_matches* out);

/* Diagnostic, no device needed: generate and compile (hiprtc, gfx950) the shape-compiled kernels of
 * representative K_seq / K_part shapes. Returns the number compiled, or -1 with the compiler log. */
int sdh_spec_selftest(char* log, size_t cap);
/* Test diagnostic: out[0] = the K_ratchet records the last push wrote, out[1] = an order-independent
 * hash of them (e2 seq, query, e1 seq), in either output mode (device records included). */
int sdh_engine_debug_digest(sdh_engine* e, uint64_t* out);
/* Diagnostic: best-of-`iters` HBM bandwidth of a streaming copy (bytes read + written) and a
 * streaming read over `bytes`-sized buffers on `device`, in GB/s -- the measured ceiling the bench
 * reports its roofline fraction against beside the 8 TB/s peak. */
int sdh_calibrate_hbm(int32_t device, int64_t bytes, int32_t iters, double* copy_gbps, double* read_gbps);
/* Library version / build info string (static storage). */
const char* sdh_version(void);
/* "src <hash> gfx950": the hash of the engine sources the library was built from
 * (siddhi_amd/csrc/src_hash.py), for checking that a deployed .so matches its source tree. */
const char* sdh_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
