/*
 * oracle.h -- CPU restatement of Siddhi's pattern/sequence engine. TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the HIP engine. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. It is never part of the product path.
 *
 * It consumes the same IR blob as libsiddhi_hip.so (siddhi_amd/ir.py) and replays the reference's
 * object graph literally (pending / newAndEvery lists of shared StateEvent objects, shallow every
 * clones, chained count slots), following org.wso2.siddhi.core.query.input.stream.state.* -- see
 * the citations in oracle.cpp.
 */
#ifndef SIDDHI_ORACLE_H
#define SIDDHI_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OracleEngine OracleEngine;

int oracle_create(const void* ir_blob, size_t len, OracleEngine** out);
/* Send n events of one stream in order. vals is row-major [n][n_attrs] of raw 64-bit attribute
 * bits (int/long sign-extended, float as its 32-bit pattern in the low word, double bits, bool 0/1,
 * string as dictionary id). nulls is [n][n_attrs] (1 = null) or NULL. Each event gets the next
 * global sequence number (0-based, in send order). as_chunk != 0 delivers the n events as one
 * Event[] chunk (single-stream receivers defer selector calls to the chunk end). */
int oracle_send(OracleEngine* e, int32_t stream, int64_t n, const int64_t* ts, const int64_t* vals,
                const uint8_t* nulls, int as_chunk);
int64_t oracle_num_matches(const OracleEngine* e);
void oracle_chm_positions(const int32_t* hashes, int64_t n, int32_t* pos);  // (test hook)
/* Total int64 words needed for the slot encoding of all matches. */
int64_t oracle_match_words(const OracleEngine* e);
/* Copy matches out in delivery order. For match i: query[i], key[i] (partition instance key id,
 * -1 if unpartitioned), ts[i]; words[off[i]..off[i+1]) encodes, per state slot, a count c followed
 * by c event sequence numbers (the slot's event chain at emission time). */
int oracle_get_matches(const OracleEngine* e, int64_t* query, int64_t* key, int64_t* ts,
                       int64_t* off, int64_t* words);
/* per match: the sequence number of the event whose processing produced it, and for an absent
 * state's timer match the instance's running max of fired times (INT64_MIN for event matches) */
int oracle_get_match_meta(const OracleEngine* e, int64_t* seq, int64_t* tb);
void oracle_clear_matches(OracleEngine* e);
/* Absent patterns' time: the runtime starts at t (SiddhiAppRuntime.start; else at the first event
 * or advance), and time passes to t with no event (the schedulers fire what falls due). */
int oracle_start(OracleEngine* e, int64_t t);
int oracle_advance_time(OracleEngine* e, int64_t t);
int oracle_set_playback(OracleEngine* e, int on);
/* String dictionary ids' text as (String.hashCode, UTF-16 length): the fan-out order of a partition
 * keyed by a string attribute hashes String.valueOf(key). */
void oracle_set_strings(OracleEngine* e, int64_t n, const int32_t* ids, const int32_t* hash, const int32_t* len);
/* Partial matches held in the pending lists of every pre-processor (after the last send). */
int64_t oracle_live_partials(const OracleEngine* e);
const char* oracle_error(const OracleEngine* e);
void oracle_destroy(OracleEngine* e);

#ifdef __cplusplus
}
#endif
#endif
